#!/bin/bash
# round 4: GPU tests on the new library (sampled dense-bucket directory keys + 8-ary locate
# steps, reciprocal bin division), then A/B of old / new / b8 (8 reads per lane per batch of
# start-only lean plans) / nokary on the small tables and full passes
OUT=gpurun_out/r4e
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $OUT/tests.log 2>&1 || { tail -60 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for v in old new b8 nokary; do
  lib=build_var/$v/librecoup_amd.so
  [ $v = new ] && lib=recoup_amd/librecoup_amd.so
  echo "== $v" >> $OUT/ab.log
  for spec in "c5 0/8" "c5 0/1" "c4 0/8" "c4 0/1" "c2 0/1"; do
    set -- $spec
    RCP_LIB_PATH=$lib CFG=$1 timeout -k 10 200 python3 tools/diag_shard_kernels.py $2 auto >> $OUT/ab.log 2>&1 || { tail $OUT/ab.log; exit 1; }
  done
done
grep -E "==|ms/pass" $OUT/ab.log
