#!/bin/bash
OUT=gpurun_out/r03e
mkdir -p $OUT
export TMPDIR=/tmp
for sh in 0/8 0/4; do
  RCP_INFLIGHT_MAX=4 timeout -k 10 300 python bench.py --no-cpu --no-e2e --sim-shard $sh > $OUT/shard_${sh/\//of}.json 2> $OUT/shard_${sh/\//of}.err || { tail $OUT/shard_${sh/\//of}.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/shard_${sh/\//of}.json')); print('$sh', round(d['ms_per_step'],4), d['config']['inflight'], d['config']['inflight_note'][-70:])"
done
for c in c5 c2 c3; do
  RCP_INFLIGHT_MAX=4 timeout -k 10 300 python bench.py --config $c --no-cpu --no-e2e > $OUT/$c.json 2> $OUT/$c.err || { tail $OUT/$c.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$c.json')); print('$c', round(d['ms_per_step'],4), d['config']['inflight'], d['config']['inflight_note'][-70:])"
done
