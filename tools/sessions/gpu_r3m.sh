#!/bin/bash
# Round-3 checkpoint on the committed tree: GPU tests, smoke, PMC traffic + C4 bench + rocprof, C2 / C3 / C5 lines
OUT=gpurun_out/r3m
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
bash tools/round_profile.sh $OUT/round > $OUT/round.log 2>&1 || { tail -30 $OUT/round.log; exit 1; }
for c in c4 c2 c3 c5; do python3 -c "
import json; d=json.load(open('$OUT/round/${c}_bench.json'))
print('$c', round(d['value']/1e9,2), 'Gbins/s', round(d['ms_per_step'],4), 'ms frac', round(d['roofline']['frac'],3), 'traffic', d['roofline']['traffic'], 'e2e', round(d['e2e']['ms'],1), 'rle', round(d['e2e']['rle_path']['ms'],1), d['e2e']['rle_path']['phases_ms'], d['e2e']['rle_path']['equal_fused'], 'parity', d['parity_sample']['ok'] if d['parity_sample'] else None)
"; done
python3 tools/kstat_rle.py $OUT/round/prof/bench_kernel_stats.csv
