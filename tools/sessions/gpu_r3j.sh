#!/bin/bash
# Heavy rows piled inside the locate kernel (no heavy launch, no slot clearing) + library memory pool:
# GPU tests, A/B vs the previous commit (base) on C4 / C5 / 1/8 shard, rocprof of the C4 bench
OUT=gpurun_out/r3j
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
BENCH_ARGS="--inflight 1" bash tools/gpu_ab.sh $OUT "c4 c5" base new base new base new || exit 1
BENCH_ARGS="--inflight 1 --sim-shard 0/8" TAG=_s8 bash tools/gpu_ab.sh $OUT "c4" base new base new || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- python3 bench.py --no-cpu --no-e2e > $OUT/c4_bench_under_rocprof.json 2> $OUT/prof.err || { tail $OUT/prof.err; exit 1; }
python3 tools/kstat_rle.py $OUT/prof/bench_kernel_stats.csv
