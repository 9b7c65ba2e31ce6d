#!/bin/bash
OUT=gpurun_out/r02w
mkdir -p $OUT
export TMPDIR=/tmp
BENCH_ARGS="--inflight 1" bash tools/gpu_ab.sh $OUT "c4 c2" ks4 base ks4 base || exit 1
BENCH_ARGS="--inflight 1 --sim-shard 0/8" TAG=_s0of8 bash tools/gpu_ab.sh $OUT "c4" ks4 base ks4 base || exit 1
