#!/bin/bash
# round 4: row-wave numerators staged in HBM (uint32) vs round-3 double staging vs LDS; locate
# without fast rows' side writes; bins kernel 16 waves; readset stall phases
OUT=gpurun_out/r4l
mkdir -p $OUT
export TMPDIR=/tmp
T="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 900 $T -m gpu tests > $OUT/tests.log 2>&1 || { tail -60 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for v in new rowsg rowslds new; do
  lib=build_var/$v/librecoup_amd.so
  [ $v = new ] && lib=recoup_amd/librecoup_amd.so
  echo "== $v" >> $OUT/c3.log
  RCP_LIB_PATH=$lib CFG=c3 timeout -k 10 200 python3 tools/diag_shard_kernels.py 0/1 auto >> $OUT/c3.log 2>&1 || { tail $OUT/c3.log; exit 1; }
done
grep -E "==|ms/pass" $OUT/c3.log
PASSES=traffic timeout -k 10 600 bash tools/pmc.sh $OUT/pmc_c3 c3 || { tail $OUT/pmc_c3/*.log; exit 1; }
python3 tools/pmc_traffic.py $OUT/pmc_c3 $OUT/traffic_c3.json profiles/fetch_calib.json || exit 1
for v in new ks2off new; do
  lib=build_var/$v/librecoup_amd.so
  [ $v = new ] && lib=recoup_amd/librecoup_amd.so
  echo "== $v" >> $OUT/ab.log
  for spec in c2:0/1 c4:0/1 c4:0/8 c5:0/8; do
    RCP_LIB_PATH=$lib CFG=${spec%%:*} timeout -k 10 200 python3 tools/diag_shard_kernels.py ${spec#*:} auto >> $OUT/ab.log 2>&1 || { tail $OUT/ab.log; exit 1; }
  done
done
grep -E "==|ms/pass" $OUT/ab.log
RCP_LIB_PATH=build_var/ptime/librecoup_amd.so STRANDED=1 timeout -k 10 300 python3 tools/diag_readset.py c5 10 > $OUT/readset_c5_phases.log 2>&1 || { tail $OUT/readset_c5_phases.log; exit 1; }
grep rep $OUT/readset_c5_phases.log
