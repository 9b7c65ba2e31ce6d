#!/bin/bash
# round 4: lean store waves 2 / 4 (default) / 6 -- C4 and C5 bench (D auto), alternating
OUT=gpurun_out/r4r
mkdir -p $OUT
export TMPDIR=/tmp
T="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread"
for rep in 1 2; do
  for v in new sw2 sw6; do
    lib=build_var/$v/librecoup_amd.so
    [ $v = new ] && lib=recoup_amd/librecoup_amd.so
    for c in c4 c5; do
      RCP_LIB_PATH=$lib timeout -k 10 300 python3 bench.py --config $c --no-cpu --no-e2e > $OUT/${v}_${c}_$rep.json 2> $OUT/${v}_${c}_$rep.err || { tail $OUT/${v}_${c}_$rep.err; exit 1; }
      python3 -c "
import json; d=json.load(open('$OUT/${v}_${c}_$rep.json')); c=d['config']
print('$v $c', round(d['ms_per_step'],4), c['inflight_note'].split('by D: ')[-1], 'kern', round(d['roofline']['kernel_ms'],4), d['inflight_check'], (d.get('parity_sample') or {}).get('equal'))"
    done
  done
done
