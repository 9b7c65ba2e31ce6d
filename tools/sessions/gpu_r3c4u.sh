#!/bin/bash
# C4 headline: start-only stream vs (start, end) pairs, same box, alternating
OUT=gpurun_out/r3c4u
mkdir -p $OUT
export TMPDIR=/tmp
BENCH_ARGS="--inflight 1" bash tools/gpu_ab.sh $OUT c4 base nouni base nouni base nouni || exit 1
