#!/bin/bash
# A/B: locate's chunk-window table read by scalar loads + per-lane select (cwsel) vs per-lane
# loads from the kernel-argument segment (base)
OUT=gpurun_out/r04z
mkdir -p $OUT
export TMPDIR=/tmp
RCP_LIB_PATH=build_var/cwsel/librecoup_amd.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/cwsel_tests.log 2>&1 || { tail -30 $OUT/cwsel_tests.log; exit 1; }
tail -1 $OUT/cwsel_tests.log
BENCH_ARGS="--inflight 1" bash tools/gpu_ab.sh $OUT "c4 c5 c2" base cwsel base cwsel
