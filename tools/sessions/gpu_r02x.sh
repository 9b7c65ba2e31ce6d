#!/bin/bash
OUT=gpurun_out/r02x
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 240 python -u -m pytest tests/test_gpu_rows.py tests/test_gpu_c3.py -x -q --timeout 120 --timeout-method thread > $OUT/rows_tests.log 2>&1 || { tail -30 $OUT/rows_tests.log; exit 1; }
tail -2 $OUT/rows_tests.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
BENCH_ARGS="--inflight 1" bash tools/gpu_ab.sh $OUT "c3" tr base tr base || exit 1
