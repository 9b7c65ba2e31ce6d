#!/bin/bash
# round 4: 1/8 shards at D > 1 -- general (auto) vs lean kernel (C4), lean vs general (C5)
OUT=gpurun_out/r4v
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
  for spec in c4:auto c4:lean c5:auto c5:general; do
    c=${spec%%:*}; k=${spec#*:}
    timeout -k 10 300 python3 bench.py --config $c --sim-shard 0/8 --kernel $k --no-cpu --no-e2e > $OUT/${c}_${k}_$rep.json 2> $OUT/${c}_${k}_$rep.err || { tail $OUT/${c}_${k}_$rep.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$OUT/${c}_${k}_$rep.json')); c=d['config']
print('$c $k', round(d['ms_per_step'],4), c['inflight_note'].split('by D: ')[-1], d['inflight_check']['equal_to_general_kernel'])"
  done
done
