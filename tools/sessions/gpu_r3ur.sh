#!/bin/bash
# start-only dense rows: one run detection for both atomics; parity, then C5 A/B
OUT=gpurun_out/r3ur
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
BENCH_ARGS="--inflight 1" bash tools/gpu_ab.sh $OUT c5 base runs2 base runs2 base runs2 || exit 1
