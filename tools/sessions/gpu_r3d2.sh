#!/bin/bash
# finer bucket directories on the latency-bound small shards (D = 1)
OUT=gpurun_out/r3d2
mkdir -p $OUT
export TMPDIR=/tmp
BENCH_ARGS="--inflight 1 --sim-shard 0/8" TAG=_s8 bash tools/gpu_ab.sh $OUT c4 base dir4 dir2 base dir4 dir2 || exit 1
BENCH_ARGS="--inflight 1" bash tools/gpu_ab.sh $OUT "c4 c2" base dir4 dir2 || exit 1
