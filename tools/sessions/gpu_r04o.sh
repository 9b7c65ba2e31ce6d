#!/bin/bash
# e2e with width runs (sorted form): C4 and C5 bench lines
OUT=gpurun_out/r04o
mkdir -p $OUT
export TMPDIR=/tmp
for c in c4 c5; do
  timeout -k 10 600 python3 bench.py --config $c --no-cpu > $OUT/${c}_bench.json 2> $OUT/${c}_bench.log || { tail $OUT/${c}_bench.log; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/${c}_bench.json')); e=d['e2e']; print('$c', round(d['ms_per_step'],4), 'e2e', round(e['ms'],1), e['phases_ms'], e['width_runs'], 'any', round(e['any_order']['ms'],1))"
done
