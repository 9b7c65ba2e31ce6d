#!/bin/bash
# lean kernel ablations (timing only): la1 no LDS adds (loads kept), la2 no output stores, la3 neither
OUT=gpurun_out/r3la
mkdir -p $OUT
export TMPDIR=/tmp
BENCH_ARGS="--inflight 1" bash tools/gpu_ab.sh $OUT "c5 c4" base la1 la2 la3 || exit 1
