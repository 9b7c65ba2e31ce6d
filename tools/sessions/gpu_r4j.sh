#!/bin/bash
# round 4: row-wave LDS staging (C3), Rle runs without a dense depth array, the r4i A/B set
# (locate ablations, decode prefetch, lean 3-buffer ring, bins-kernel waves), readset stalls
OUT=gpurun_out/r4j
mkdir -p $OUT
export TMPDIR=/tmp
T="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 300 $T -m gpu tests/test_gpu_rows.py tests/test_gpu_rle.py > $OUT/rows_rle.log 2>&1 || { tail -60 $OUT/rows_rle.log; exit 1; }
tail -1 $OUT/rows_rle.log
for v in new rowsg rows12; do
  lib=build_var/$v/librecoup_amd.so
  [ $v = new ] && lib=recoup_amd/librecoup_amd.so
  echo "== $v" >> $OUT/c3.log
  RCP_LIB_PATH=$lib CFG=c3 timeout -k 10 200 python3 tools/diag_shard_kernels.py 0/1 auto general >> $OUT/c3.log 2>&1 || { tail $OUT/c3.log; exit 1; }
done
grep -E "==|ms/pass" $OUT/c3.log
PASSES=traffic timeout -k 10 600 bash tools/pmc.sh $OUT/pmc_c3 c3 || { tail $OUT/pmc_c3/*.log; exit 1; }
python3 tools/pmc_traffic.py $OUT/pmc_c3 $OUT/traffic_c3.json profiles/fetch_calib.json || exit 1
for v in new covdense; do
  lib=build_var/$v/librecoup_amd.so
  [ $v = new ] && lib=recoup_amd/librecoup_amd.so
  RCP_LIB_PATH=$lib ITERS=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/rle_$v -o p -- python3 tools/prof_rle.py c4 > $OUT/rle_$v.log 2>&1 || { tail $OUT/rle_$v.log; exit 1; }
  grep -E "iter|equal" $OUT/rle_$v.log
  python3 tools/kstat_rle.py $OUT/rle_$v/p_kernel_stats.csv
done
timeout -k 10 900 $T -m gpu tests > $OUT/tests.log 2>&1 || { tail -60 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
STRANDED=1 timeout -k 10 300 python3 tools/diag_readset.py c5 12 > $OUT/readset_c5.log 2>&1 || { tail $OUT/readset_c5.log; exit 1; }
grep rep $OUT/readset_c5.log
RCP_LIB_PATH=build_var/pool200/librecoup_amd.so STRANDED=1 timeout -k 10 300 python3 tools/diag_readset.py c5 12 > $OUT/readset_c5_pool200.log 2>&1 || { tail $OUT/readset_c5_pool200.log; exit 1; }
grep rep $OUT/readset_c5_pool200.log
for v in new ks2off wpe5 nopre l1 l2 l4 l8; do
  lib=build_var/$v/librecoup_amd.so
  [ $v = new ] && lib=recoup_amd/librecoup_amd.so
  echo "== $v" >> $OUT/ab.log
  specs="c2:0/1 c4:0/1"
  case $v in new|nopre) specs="c2:0/1 c4:0/1 c4:0/8 c5:0/8";; ks2off|wpe5) specs="c2:0/1 c4:0/1 c4:0/8";; esac
  for spec in $specs; do
    RCP_LIB_PATH=$lib CFG=${spec%%:*} timeout -k 10 200 python3 tools/diag_shard_kernels.py ${spec#*:} auto >> $OUT/ab.log 2>&1 || { tail $OUT/ab.log; exit 1; }
  done
done
for v in ring3 ring3b8; do
  echo "== $v" >> $OUT/ab.log
  for spec in c5:0/8 c5:0/1 c4:0/1; do
    RCP_LIB_PATH=build_var/$v/librecoup_amd.so CFG=${spec%%:*} timeout -k 10 200 python3 tools/diag_shard_kernels.py ${spec#*:} auto >> $OUT/ab.log 2>&1 || { tail $OUT/ab.log; exit 1; }
  done
done
for v in bd8 bd16; do
  echo "== $v" >> $OUT/ab.log
  RCP_LIB_PATH=build_var/$v/librecoup_amd.so CFG=c2 timeout -k 10 200 python3 tools/diag_shard_kernels.py 0/1 auto >> $OUT/ab.log 2>&1 || { tail $OUT/ab.log; exit 1; }
done
echo "== kernels" >> $OUT/ab.log
CFG=c5 timeout -k 10 200 python3 tools/diag_shard_kernels.py 0/8 auto general rows >> $OUT/ab.log 2>&1 || { tail $OUT/ab.log; exit 1; }
CFG=c4 timeout -k 10 200 python3 tools/diag_shard_kernels.py 0/8 auto lean rows >> $OUT/ab.log 2>&1 || { tail $OUT/ab.log; exit 1; }
grep -E "==|ms/pass" $OUT/ab.log
