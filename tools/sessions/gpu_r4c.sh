#!/bin/bash
# round 4: full GPU test suite, default bench, then the shard baseline (gpu_r4a.sh)
OUT=gpurun_out/r4c
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > $OUT/tests.log 2>&1 || { tail -60 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
timeout -k 10 400 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'],d['ms_per_step'],d['config']['single_pass_ms'],d['inflight_check'],d['cpu_baseline']['value'],d['cpu_baseline']['one_core'],d['parity_sample'])"
bash tools/sessions/gpu_r4a.sh
