#!/bin/bash
# round 4: one-round general kernel for small tables -- GPU suite, C4 shard + C2 / C3 lines
OUT=gpurun_out/r4zc
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $OUT/tests.log 2>&1 || { tail -60 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for spec in c4:0/8 c5:0/8; do
  timeout -k 10 300 python3 bench.py --config ${spec%%:*} --sim-shard ${spec#*:} --no-cpu --no-e2e > $OUT/shard_${spec%%:*}.json 2> $OUT/shard_${spec%%:*}.err || { tail $OUT/shard_${spec%%:*}.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/shard_${spec%%:*}.json')); c=d['config']
print('$spec', round(d['ms_per_step'],4), c['inflight_note'].split('by D: ')[-1], d['inflight_check']['equal_to_general_kernel'])"
done
