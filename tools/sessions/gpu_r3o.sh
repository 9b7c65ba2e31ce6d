#!/bin/bash
# Locate side outputs only where read (lean plans): GPU tests, A/B vs base on C4 / C5 / 1/8 shard
OUT=gpurun_out/r3o
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
BENCH_ARGS="--inflight 1" bash tools/gpu_ab.sh $OUT "c4 c5" base side base side base side || exit 1
BENCH_ARGS="--inflight 1 --sim-shard 0/8" TAG=_s8 bash tools/gpu_ab.sh $OUT "c4" base side base side || exit 1
