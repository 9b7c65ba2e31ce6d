#!/bin/bash
# uniform-width reads: the lean kernel streams starts alone; GPU suite, C4 / C5 lines, rocprof
OUT=gpurun_out/r3u2
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
for c in c4 c5; do
timeout -k 10 600 python3 bench.py --config $c --no-cpu --no-e2e > $OUT/$c.json 2> $OUT/$c.err || { tail $OUT/$c.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/$c.json')); print('$c', round(d['ms_per_step'],4), 'single', round(d['config']['single_pass_ms'],4), {k: round(v,4) for k,v in d['kernel_ms'].items()}, 'frac', round(d['roofline']['frac'],3))"
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o p -- python3 bench.py --no-cpu --no-e2e --inflight 1 > $OUT/c4_rocprof.json 2> $OUT/prof.err || { tail $OUT/prof.err; exit 1; }
python3 -c "
import csv
for r in csv.DictReader(open('$OUT/prof/p_kernel_stats.csv')):
    if any(k in r['Name'] for k in ('lean','locate','heavy')): print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1000,1), 'us')
"
