#!/bin/bash
# r02 final profiles: rocprof kernel stats (C4, C3), PMC traffic per config keyed by kernel, bench lines
OUT=gpurun_out/r02t
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c4 -o bench -- \
    python3 bench.py --no-cpu --no-e2e > $OUT/c4_bench_under_rocprof.json 2> $OUT/prof_c4.err || { tail $OUT/prof_c4.err; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c3 -o bench -- \
    python3 bench.py --config c3 --no-cpu --no-e2e > $OUT/c3_bench_under_rocprof.json 2> $OUT/prof_c3.err || { tail $OUT/prof_c3.err; exit 1; }
for c in c4 c5 c2 c3; do
  PASSES=traffic timeout -k 10 400 bash tools/pmc.sh $OUT/pmc_$c $c || { echo "pmc $c failed"; exit 1; }
  python3 tools/pmc_traffic.py $OUT/pmc_$c $OUT/traffic_$c.json profiles/fetch_calib.json > /dev/null || exit 1
done
for c in c4 c5 c2 c3; do python3 -c "import json; d=json.load(open('$OUT/traffic_$c.json')); print('$c', d['kernel'], round(d['hbm_bytes_per_launch']/1e9,4), 'GB')"; done
for c in c5 c2 c3 c4; do
  timeout -k 10 600 python3 bench.py --config $c --traffic $OUT/traffic_$c.json > $OUT/${c}_bench.json 2> $OUT/${c}_bench.err || { tail $OUT/${c}_bench.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/${c}_bench.json')); print('$c', round(d['ms_per_step'],4), '%.3e' % d['value'], d['config']['inflight'], d['roofline']['frac'], d['roofline']['traffic'], d['parity_sample'])"
done
find $OUT/prof_c4 $OUT/prof_c3 -name "*kernel_stats.csv" | while read f; do echo "== $f"; python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    if 'rcp_' in r['Name']: print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,2), 'us')
"; done
