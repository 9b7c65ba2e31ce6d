#!/bin/bash
# round 4: coverage (Rle) pileup rounds per workgroup 1 / 2 (new) / 4 -- C4 kernel times
OUT=gpurun_out/r4x
mkdir -p $OUT
export TMPDIR=/tmp
T="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 600 $T -m gpu tests > $OUT/tests.log 2>&1 || { tail -60 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for v in csr1 csr4; do
  RCP_LIB_PATH=build_var/$v/librecoup_amd.so timeout -k 10 300 $T -m gpu tests/test_gpu_rle.py > $OUT/rle_$v.log 2>&1 || { tail -30 $OUT/rle_$v.log; exit 1; }
  echo "$v $(tail -1 $OUT/rle_$v.log)"
done
for v in new csr1 csr4; do
  lib=build_var/$v/librecoup_amd.so
  [ $v = new ] && lib=recoup_amd/librecoup_amd.so
  RCP_LIB_PATH=$lib ITERS=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/rle_$v -o p -- python3 tools/prof_rle.py c4 > $OUT/rle_$v.txt 2>&1 || { tail $OUT/rle_$v.txt; exit 1; }
  echo "== $v"; grep -E "equal" $OUT/rle_$v.txt
  python3 tools/kstat_rle.py $OUT/rle_$v/p_kernel_stats.csv | grep -E "pileup_kernel<false, true|cov_runs"
done
# heavy grid scaled by the table's rows (hg32) vs 4096 blocks always (new)
for v in new hg32 new hg32; do
  lib=build_var/$v/librecoup_amd.so
  [ $v = new ] && lib=recoup_amd/librecoup_amd.so
  echo "== $v" >> $OUT/hg.log
  for spec in c4:0/8 c5:0/8 c4:0/1; do
    RCP_LIB_PATH=$lib CFG=${spec%%:*} timeout -k 10 200 python3 tools/diag_shard_kernels.py ${spec#*:} auto >> $OUT/hg.log 2>&1 || { tail $OUT/hg.log; exit 1; }
  done
done
grep -E "==|ms/pass" $OUT/hg.log
