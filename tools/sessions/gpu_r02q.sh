#!/bin/bash
OUT=gpurun_out/r02q
mkdir -p $OUT
export TMPDIR=/tmp
BENCH_ARGS="--inflight 1" bash tools/gpu_ab.sh $OUT "c3" base nostore rowmajor base nostore rowmajor || exit 1
