#!/bin/bash
# round 4: C4 1/8 shard bench (D auto) with one general round (new) vs two (g2), alternating
OUT=gpurun_out/r4zd
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2 3; do
  for v in new g2; do
    lib=build_var/$v/librecoup_amd.so
    [ $v = new ] && lib=recoup_amd/librecoup_amd.so
    RCP_LIB_PATH=$lib timeout -k 10 300 python3 bench.py --config c4 --sim-shard 0/8 --no-cpu --no-e2e > $OUT/${v}_$rep.json 2> $OUT/${v}_$rep.err || { tail $OUT/${v}_$rep.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$OUT/${v}_$rep.json')); c=d['config']
print('$v', round(d['ms_per_step'],4), c['inflight_note'].split('by D: ')[-1], round(d['roofline']['kernel_ms'],4))"
  done
done
