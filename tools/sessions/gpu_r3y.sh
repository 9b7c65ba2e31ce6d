#!/bin/bash
# round-3 checkpoint 2: GPU suite + smoke, the measurement set (PMC traffic, C4 line, rocprof
# summary, C2 / C3 / C5 lines), the 1/8 and 1/4 C4 shard rehearsals
OUT=gpurun_out/r3y
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail $OUT/smoke.log; exit 1; }
bash tools/round_profile.sh $OUT > $OUT/round.log 2>&1 || { tail -20 $OUT/round.log; exit 1; }
for s in 0/8 0/4; do
n=$(echo $s | tr / o)
timeout -k 10 300 python3 bench.py --sim-shard $s --no-cpu --no-e2e > $OUT/shard_$n.json 2> $OUT/shard_$n.err || { tail $OUT/shard_$n.err; exit 1; }
done
for f in c4 c2 c3 c5; do python3 -c "import json; d=json.load(open('$OUT/${f}_bench.json')); print('$f', round(d['value']/1e9,1), 'Grb/s', round(d['ms_per_step'],4), 'ms', 'frac', round(d['roofline']['frac'],3), 'single', round(d['config']['single_pass_ms'],4), 'e2e', d.get('e2e',{}).get('ms') if isinstance(d.get('e2e'),dict) else None)"; done
for n in 0o8 0o4; do python3 -c "import json; d=json.load(open('$OUT/shard_$n.json')); print('$n', round(d['ms_per_step'],4), round(d['config']['single_pass_ms'],4))"; done
