#!/bin/bash
OUT=gpurun_out/r03c
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
BENCH_ARGS="--inflight 1" bash tools/gpu_ab.sh $OUT "c3" prev base prev base || exit 1
