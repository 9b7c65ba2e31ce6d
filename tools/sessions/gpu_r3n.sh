#!/bin/bash
# A/B general kernel rounds per workgroup 2 (base) vs 1 on C2 (10k TSS rows, 20-bp bins)
OUT=gpurun_out/r3n
mkdir -p $OUT
export TMPDIR=/tmp
BENCH_ARGS="--inflight 1" bash tools/gpu_ab.sh $OUT "c2" r2 r1 r2 r1 r2 r1 || exit 1
