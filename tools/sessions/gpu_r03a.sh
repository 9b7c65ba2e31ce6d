#!/bin/bash
OUT=gpurun_out/r03a
mkdir -p $OUT
export TMPDIR=/tmp
BENCH_ARGS="--inflight 1" bash tools/gpu_ab.sh $OUT "c3" noruns runs8 runs4 noruns runs8 runs4 || exit 1
