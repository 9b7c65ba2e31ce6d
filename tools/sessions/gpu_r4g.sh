#!/bin/bash
# round 4: GPU tests (16 column chunks, per-base shard split, linear final locate pass), A/B of
# new / lin0 (bisection only) / lin32 / nosplit on the small tables and full passes
OUT=gpurun_out/r4g
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $OUT/tests.log 2>&1 || { tail -60 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for v in new lin0 lin32 nosplit; do
  lib=build_var/$v/librecoup_amd.so
  [ $v = new ] && lib=recoup_amd/librecoup_amd.so
  echo "== $v" >> $OUT/ab.log
  for spec in "c5 0/8" "c5 7/8" "c5 0/1" "c4 0/8" "c4 0/1" "c2 0/1"; do
    set -- $spec
    RCP_LIB_PATH=$lib CFG=$1 timeout -k 10 200 python3 tools/diag_shard_kernels.py $2 auto >> $OUT/ab.log 2>&1 || { tail $OUT/ab.log; exit 1; }
  done
done
grep -E "==|ms/pass" $OUT/ab.log
# the R path's host side: D2H destinations with / without the huge-page hint
for k in 1 2; do
  RCP_NO_THP_ADVISE=1 ITERS=3 timeout -k 10 300 python3 tools/prof_rle.py c4 >> $OUT/rle.log 2>&1 || { tail $OUT/rle.log; exit 1; }
  echo "-- advise" >> $OUT/rle.log
  ITERS=3 timeout -k 10 300 python3 tools/prof_rle.py c4 >> $OUT/rle.log 2>&1 || { tail $OUT/rle.log; exit 1; }
done
grep -E "iter|advise" $OUT/rle.log
