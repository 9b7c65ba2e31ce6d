#!/bin/bash
# round 4: e2e / rle_path with the host runs released between calls (C4, C5)
OUT=gpurun_out/r4u
mkdir -p $OUT
export TMPDIR=/tmp
for c in c4 c5; do
  timeout -k 10 500 python3 bench.py --config $c --no-cpu > $OUT/$c.json 2> $OUT/$c.err || { tail $OUT/$c.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/$c.json')); e=d['e2e']
print('$c', round(e['ms'],1), e['phases_ms'], 'rle', round(e['rle_path']['ms'],1), e['rle_path']['phases_ms'], e['rle_path']['calls_ms'], e['rle_path']['equal_fused'])"
done
