#!/bin/bash
# general pileup kernel ablations on C2 and the 1/8 C4 shard: no stores / no reads / neither
OUT=gpurun_out/r3u
mkdir -p $OUT
export TMPDIR=/tmp
bash tools/gpu_ab.sh $OUT c2 base nost nord none && BENCH_ARGS="--sim-shard 0/8 --inflight 1" TAG=_s8 bash tools/gpu_ab.sh $OUT c4 base nost nord none
