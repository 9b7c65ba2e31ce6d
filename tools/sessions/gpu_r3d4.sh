#!/bin/bash
# four distinct samples in flight vs three
OUT=gpurun_out/r3d4
mkdir -p $OUT
export TMPDIR=/tmp
for c in c2 c3 c5 c4; do
for d in 3 4 3 4; do
timeout -k 10 600 python3 bench.py --config $c --no-cpu --no-e2e --inflight $d > $OUT/${c}_$d.json 2> $OUT/${c}_$d.err || { tail $OUT/${c}_$d.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/${c}_$d.json')); print('$c D=$d', round(d['ms_per_step'],4))"
done
done
