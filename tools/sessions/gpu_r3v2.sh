#!/bin/bash
# start-only stream everywhere: the widened tests, and C2's bench parity sample (general kernel)
OUT=gpurun_out/r3v2
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_lean.py tests/test_gpu_rle.py tests/test_gpu_configs.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 600 python3 bench.py --config c2 --no-e2e > $OUT/c2.json 2> $OUT/c2.err || { tail $OUT/c2.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/c2.json')); print('c2', d['ms_per_step'], d['parity_sample'])"
