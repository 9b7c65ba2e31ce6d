#!/bin/bash
# A/B: directory buckets of ~8 (base), ~4 and ~2 mean reads: locate time vs pileup, C4 / C2 / C5
OUT=gpurun_out/r3f
mkdir -p $OUT
export TMPDIR=/tmp
BENCH_ARGS="--inflight 1" bash tools/gpu_ab.sh $OUT "c4 c2 c5" base dir4 dir2 base dir4 dir2
grep -h "readset + plan" $OUT/*.err
