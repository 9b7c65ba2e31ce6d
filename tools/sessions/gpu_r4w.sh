#!/bin/bash
# round 4: row-wave HBM stage with two 8-wave workgroups per CU (rw8) vs one 16-wave (new), C3
OUT=gpurun_out/r4w
mkdir -p $OUT
export TMPDIR=/tmp
T="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread"
RCP_LIB_PATH=build_var/rw8/librecoup_amd.so timeout -k 10 300 $T -m gpu tests/test_gpu_rows.py > $OUT/rows_rw8.log 2>&1 || { tail -30 $OUT/rows_rw8.log; exit 1; }
echo "rw8 $(tail -1 $OUT/rows_rw8.log)"
for v in new rw8 new rw8; do
  lib=build_var/$v/librecoup_amd.so
  [ $v = new ] && lib=recoup_amd/librecoup_amd.so
  echo "== $v" >> $OUT/c3.log
  RCP_LIB_PATH=$lib CFG=c3 timeout -k 10 200 python3 tools/diag_shard_kernels.py 0/1 auto >> $OUT/c3.log 2>&1 || { tail $OUT/c3.log; exit 1; }
done
grep -E "==|ms/pass" $OUT/c3.log
