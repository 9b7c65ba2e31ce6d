#!/bin/bash
# general kernel occupancy at C4 shapes: stage of <= 256 bins (two workgroups per CU) or a
# single-buffered stage, vs base; 1/8 and 1/4 C4 shards (general kernel) and full C4 (lean)
OUT=gpurun_out/r3g
mkdir -p $OUT
export TMPDIR=/tmp
BENCH_ARGS="--inflight 1 --sim-shard 0/8" TAG=_s8 bash tools/gpu_ab.sh $OUT c4 base sb256 buf1 base sb256 buf1 || exit 1
BENCH_ARGS="--inflight 1 --sim-shard 0/4" TAG=_s4 bash tools/gpu_ab.sh $OUT c4 base sb256 buf1 || exit 1
BENCH_ARGS="--inflight 1" bash tools/gpu_ab.sh $OUT "c4 c2" base sb256 buf1 || exit 1
