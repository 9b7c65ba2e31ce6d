#!/bin/bash
# rocprof kernel stats of the bench command (C4 and the 1/8 shard), PMC traffic per config
OUT=gpurun_out/r02d
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c4 -o bench -- \
    python3 bench.py --no-cpu --no-e2e > $OUT/c4_bench_under_rocprof.json 2> $OUT/prof_c4.err || { tail $OUT/prof_c4.err; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_s08 -o bench -- \
    python3 bench.py --no-cpu --no-e2e --sim-shard 0/8 > $OUT/s08_bench_under_rocprof.json 2> $OUT/prof_s08.err || { tail $OUT/prof_s08.err; exit 1; }
for c in c4 c5 c2 c3; do
  PASSES=traffic timeout -k 10 400 bash tools/pmc.sh $OUT/pmc_$c $c || { echo "pmc $c failed"; exit 1; }
  python3 tools/pmc_traffic.py $OUT/pmc_$c $OUT/traffic_$c.json profiles/fetch_calib.json > /dev/null || exit 1
done
for c in c4 c5 c2 c3; do python3 -c "import json; d=json.load(open('$OUT/traffic_$c.json')); print('$c', d['kernel'], round(d['hbm_bytes_per_launch']/1e9,4), 'GB')"; done
find $OUT/prof_c4 $OUT/prof_s08 -name "*kernel_stats.csv" | while read f; do echo "== $f"; python3 -c "
import csv,sys
for r in csv.DictReader(open('$f')):
    if 'rcp_' in r['Name']: print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,2), 'us')
"; done
