#!/bin/bash
# C5 line after the shared run detection (PMC traffic + bench with CPU baseline and e2e)
OUT=gpurun_out/r3c5
mkdir -p $OUT
export TMPDIR=/tmp
PASSES=traffic bash tools/pmc.sh $OUT/pmc_c5 c5 || exit 1
python3 tools/pmc_traffic.py $OUT/pmc_c5 $OUT/traffic_c5.json profiles/fetch_calib.json > /dev/null || exit 1
timeout -k 10 600 python3 bench.py --config c5 --traffic $OUT/traffic_c5.json > $OUT/c5_bench.json 2> $OUT/c5_bench.err || { tail $OUT/c5_bench.err; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- python3 bench.py --config c5 --no-cpu --no-e2e --inflight 1 --traffic $OUT/traffic_c5.json > $OUT/c5_bench_under_rocprof.json 2> $OUT/prof.err || { tail $OUT/prof.err; exit 1; }
python3 - <<'PY'
import csv, json
d = json.load(open('gpurun_out/r3c5/c5_bench.json'))
r = d['roofline']; e = d['e2e']
print('c5', round(d['ms_per_step'], 4), d['config']['inflight_note'][-60:], 'frac', round(r['frac'], 3), 'traffic', r['traffic'], 'kernel_ms', r['kernel_ms'], 'e2e', round(e['ms'], 1), 'parity', d['parity_sample'])
for row in csv.DictReader(open('gpurun_out/r3c5/prof/bench_kernel_stats.csv')):
    if any(k in row['Name'] for k in ('lean', 'locate', 'heavy')): print(row['Name'][:60], row['Calls'], round(float(row['AverageNs']) / 1000, 1), 'us')
PY
