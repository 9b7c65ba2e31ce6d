#!/bin/bash
OUT=gpurun_out/r02v
mkdir -p $OUT
export TMPDIR=/tmp
BENCH_ARGS="--inflight 1" bash tools/gpu_ab.sh $OUT "c3" base rmnt t128 both base rmnt t128 both || exit 1
