#!/bin/bash
OUT=gpurun_out/r02o
mkdir -p $OUT
export TMPDIR=/tmp
for c in c2 c5 c4; do
  timeout -k 10 600 python bench.py --config $c --no-cpu --no-e2e > $OUT/${c}_bench.json 2> $OUT/${c}_bench.err || { tail $OUT/${c}_bench.err; exit 1; }
done
for sh in 0/8 0/4 0/2; do
  timeout -k 10 300 python bench.py --no-cpu --no-e2e --sim-shard $sh > $OUT/shard_${sh/\//of}.json 2> $OUT/shard_${sh/\//of}.err || { tail $OUT/shard_${sh/\//of}.err; exit 1; }
done
for f in $OUT/*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', round(d['ms_per_step'],4), '%.3e' % d['value'], d['config']['inflight'], d['config']['inflight_note'][-60:])"; done
