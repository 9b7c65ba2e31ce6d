#!/bin/bash
# round 4: row-wave HBM numerator stage with enlarged-bin masks (new), fp64 stage (s3), 6 slots
OUT=gpurun_out/r4n
mkdir -p $OUT
export TMPDIR=/tmp
T="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 600 $T -m gpu tests > $OUT/tests.log 2>&1 || { tail -60 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for v in s3 sl6; do
  RCP_LIB_PATH=build_var/$v/librecoup_amd.so timeout -k 10 300 $T -m gpu tests/test_gpu_rows.py > $OUT/rows_$v.log 2>&1 || { tail -40 $OUT/rows_$v.log; exit 1; }
  echo "$v $(tail -1 $OUT/rows_$v.log)"
done
for v in new s3 sl6 new s3 sl6; do
  lib=build_var/$v/librecoup_amd.so
  [ $v = new ] && lib=recoup_amd/librecoup_amd.so
  echo "== $v" >> $OUT/c3.log
  RCP_LIB_PATH=$lib CFG=c3 timeout -k 10 200 python3 tools/diag_shard_kernels.py 0/1 auto >> $OUT/c3.log 2>&1 || { tail $OUT/c3.log; exit 1; }
done
grep -E "==|ms/pass" $OUT/c3.log
for v in new sl6; do
  lib=build_var/$v/librecoup_amd.so
  [ $v = new ] && lib=recoup_amd/librecoup_amd.so
  RCP_LIB_PATH=$lib PASSES=traffic timeout -k 10 600 bash tools/pmc.sh $OUT/pmc_$v c3 || { tail $OUT/pmc_$v/*.log; exit 1; }
  python3 tools/pmc_traffic.py $OUT/pmc_$v $OUT/traffic_$v.json profiles/fetch_calib.json | grep -E "hbm_bytes|fetch_bytes|write_bytes" || exit 1
done
