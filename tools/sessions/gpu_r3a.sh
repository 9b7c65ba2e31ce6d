#!/bin/bash
# Round 3 start: GPU tests, smoke, default bench line, rocprof summary of the C4 bench
OUT=gpurun_out/r3a
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
timeout -k 10 400 python bench.py > $OUT/c4_bench.json 2> $OUT/c4_bench.err || { tail $OUT/c4_bench.err; exit 1; }
cat $OUT/c4_bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- python3 bench.py --no-cpu --no-e2e > $OUT/c4_bench_under_rocprof.json 2> $OUT/prof.err || { tail $OUT/prof.err; exit 1; }
find $OUT/prof -name '*kernel_stats.csv' | head -3
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_rle -o rle -- python3 tools/prof_rle.py c4 > $OUT/prof_rle_c4.log 2>&1 || { tail $OUT/prof_rle_c4.log; exit 1; }
cat $OUT/prof_rle_c4.log
