#!/bin/bash
OUT=gpurun_out/r02k
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 600 python bench.py > $OUT/c4_bench.json 2> $OUT/c4_bench.err || { tail $OUT/c4_bench.err; exit 1; }
cat $OUT/c4_bench.json
