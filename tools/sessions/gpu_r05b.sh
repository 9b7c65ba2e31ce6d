#!/bin/bash
# A/B: row-wave staging as 32-bit numerators (num32) vs 8-B means (base); GPU tests on num32
OUT=gpurun_out/r05b
mkdir -p $OUT
export TMPDIR=/tmp
RCP_LIB_PATH=build_var/num32/librecoup_amd.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/num32_tests.log 2>&1 || { tail -30 $OUT/num32_tests.log; exit 1; }
tail -1 $OUT/num32_tests.log
BENCH_ARGS="--inflight 1" bash tools/gpu_ab.sh $OUT c3 base num32 base num32 base num32
