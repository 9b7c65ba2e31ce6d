#!/bin/bash
OUT=gpurun_out/r02z
mkdir -p $OUT
export TMPDIR=/tmp
BENCH_ARGS="--inflight 1" bash tools/gpu_ab.sh $OUT "c3" base noatomic base noatomic || exit 1
