#!/bin/bash
# A/B repeat (cwsel vs base), C4 and C2, three alternations
OUT=gpurun_out/r04z2
mkdir -p $OUT
export TMPDIR=/tmp
BENCH_ARGS="--inflight 1" bash tools/gpu_ab.sh $OUT "c4 c2" base cwsel base cwsel base cwsel
