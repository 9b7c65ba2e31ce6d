#!/bin/bash
# Sanity pass of the committed tree on a fresh box: GPU tests, smoke, default bench line, C3 line
OUT=gpurun_out/r02e
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -3 $OUT/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail $OUT/smoke.log; exit 1; }
timeout -k 10 600 python bench.py > $OUT/c4_bench.json 2> $OUT/c4_bench.err || { tail $OUT/c4_bench.err; exit 1; }
cat $OUT/c4_bench.json
timeout -k 10 600 python bench.py --config c3 > $OUT/c3_bench.json 2> $OUT/c3_bench.err || { tail $OUT/c3_bench.err; exit 1; }
cat $OUT/c3_bench.json
