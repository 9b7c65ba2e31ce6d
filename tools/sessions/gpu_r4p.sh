#!/bin/bash
# round 4: lean persistent grid taking 6/8, 7/8 of the workgroup slots (room for the next
# sample's locate + heavy) vs all of them, C4 bench with samples in flight, alternating
OUT=gpurun_out/r4p
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
  for v in new f6 f7; do
    lib=build_var/$v/librecoup_amd.so
    [ $v = new ] && lib=recoup_amd/librecoup_amd.so
    RCP_LIB_PATH=$lib timeout -k 10 300 python3 bench.py --no-cpu --no-e2e > $OUT/${v}_$rep.json 2> $OUT/${v}_$rep.err || { tail $OUT/${v}_$rep.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$OUT/${v}_$rep.json')); c=d['config']
print('$v', round(d['ms_per_step'],4), c['inflight'], c['inflight_note'].split(': ')[-1], round(d['roofline']['kernel_ms'],4))"
  done
done
