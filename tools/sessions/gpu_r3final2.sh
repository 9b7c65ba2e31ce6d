#!/bin/bash
# round-3 final measurement set: GPU suite + smoke, PMC traffic (C4, C5), the C4 line with it,
# rocprof summary, C2 / C3 / C5 lines, 1/8 and 1/4 shard rehearsals
OUT=gpurun_out/r3final2
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail $OUT/smoke.log; exit 1; }
PASSES=traffic bash tools/pmc.sh $OUT/pmc_c5 c5 || exit 1
python3 tools/pmc_traffic.py $OUT/pmc_c5 $OUT/traffic_c5.json || exit 1
bash tools/round_profile.sh $OUT > $OUT/round.log 2>&1 || { tail -20 $OUT/round.log; exit 1; }
timeout -k 10 600 python3 bench.py --config c5 --traffic $OUT/traffic_c5.json > $OUT/c5_bench.json 2> $OUT/c5_bench.err || { tail $OUT/c5_bench.err; exit 1; }
for s in 0/8 0/4; do
n=$(echo $s | tr / o)
timeout -k 10 300 python3 bench.py --sim-shard $s --no-cpu --no-e2e > $OUT/shard_$n.json 2> $OUT/shard_$n.err || { tail $OUT/shard_$n.err; exit 1; }
done
for f in c4 c2 c3 c5; do python3 -c "import json; d=json.load(open('$OUT/${f}_bench.json')); r=d['roofline']; print('$f', round(d['value']/1e9,1), 'Grb/s', round(d['ms_per_step'],4), 'ms single', round(d['config']['single_pass_ms'],4), 'frac', round(r['frac'],3), 'traffic', r['traffic'], 'e2e', round(d['e2e']['ms'],1) if isinstance(d.get('e2e'),dict) else None)"; done
for n in 0o8 0o4; do python3 -c "import json; d=json.load(open('$OUT/shard_$n.json')); print('$n', round(d['ms_per_step'],4), round(d['config']['single_pass_ms'],4))"; done
