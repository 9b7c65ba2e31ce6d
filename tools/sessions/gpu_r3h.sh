#!/bin/bash
# A/B locate: heavy-slot clearing after the rows (base) vs before (first); ablations abl1 (no side writes), abl2 (no bucket searches)
OUT=gpurun_out/r3h
mkdir -p $OUT
export TMPDIR=/tmp
BENCH_ARGS="--inflight 1" bash tools/gpu_ab.sh $OUT "c4 c2" base first abl1 abl2 base first abl1 abl2
