#!/bin/bash
# round 4: the bin-difference kernel -- its tests, the whole GPU suite, C2 timing against the general kernel
OUT=gpurun_out/r4f
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_bins.py > $OUT/bins_tests.log 2>&1 || { tail -60 $OUT/bins_tests.log; exit 1; }
tail -3 $OUT/bins_tests.log
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $OUT/tests.log 2>&1 || { tail -60 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
CFG=c2 timeout -k 10 200 python3 tools/diag_shard_kernels.py 0/1 auto general >> $OUT/ab.log 2>&1 || { tail $OUT/ab.log; exit 1; }
CFG=c2 timeout -k 10 200 python3 tools/diag_shard_kernels.py 0/1 auto general >> $OUT/ab.log 2>&1 || { tail $OUT/ab.log; exit 1; }
grep ms/pass $OUT/ab.log
