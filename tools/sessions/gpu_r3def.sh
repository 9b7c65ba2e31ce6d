#!/bin/bash
# the driver's default bench command (N=1), twice, and smoke
OUT=gpurun_out/r3def
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail $OUT/smoke.log; exit 1; }
for k in 1 2; do
timeout -k 10 900 python3 bench.py > $OUT/bench_$k.json 2> $OUT/bench_$k.err || { tail $OUT/bench_$k.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench_$k.json')); print(d['value'], d['ms_per_step'], d['config']['inflight_note'][-80:], d['roofline']['frac'], d['parity_sample']['ok'])"
done
