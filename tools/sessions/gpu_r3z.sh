#!/bin/bash
# interpolation / wide-median rows piled as one pair stream split over the block's waves
OUT=gpurun_out/r3z
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 600 python3 bench.py --config c3 --no-cpu --no-e2e --inflight 1 > $OUT/c3_bench.json 2> $OUT/c3_bench.err || { tail $OUT/c3_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/c3_bench.json')); print('c3', round(d['ms_per_step'],4), d['kernel_ms'])"
