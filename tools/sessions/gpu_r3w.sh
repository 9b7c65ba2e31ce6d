#!/bin/bash
# default build after the per-base two-round lean items: GPU suite, C5 bench line
OUT=gpurun_out/r3w
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 600 python3 bench.py --config c5 --no-cpu > $OUT/c5_bench.json 2> $OUT/c5_bench.err || { tail $OUT/c5_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/c5_bench.json')); print('c5', d['value'], d['ms_per_step'], d['config'].get('inflight_note'), d['roofline']['frac'], d['single_pass_ms'] if 'single_pass_ms' in d else d['config'].get('single_pass_ms'))"
