#!/bin/bash
# round 4: concurrent plans in the bench (D > 1) -- full GPU suite, C4 / C5 / C2 bench lines
OUT=gpurun_out/r4q
mkdir -p $OUT
export TMPDIR=/tmp
T="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 600 $T -m gpu tests > $OUT/tests.log 2>&1 || { tail -60 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for c in c4 c4 c5 c2 c3; do
  timeout -k 10 300 python3 bench.py --config $c --no-cpu --no-e2e > $OUT/${c}.json 2> $OUT/${c}.err || { tail $OUT/${c}.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/${c}.json')); c=d['config']
print('$c', d['value'], round(d['ms_per_step'],4), c['inflight_note'].split('by D: ')[-1], 'check', d['inflight_check'])"
done
