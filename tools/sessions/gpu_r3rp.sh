#!/bin/bash
# rocprof summary of single-pass C4 launches (--inflight 1: the D tuning's concurrent passes
# inflate per-kernel durations) and the bench line beside it
OUT=gpurun_out/r3rp
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- \
    python3 bench.py --no-cpu --no-e2e --inflight 1 --traffic gpurun_out/r3final/traffic_c4.json > $OUT/c4_bench_under_rocprof.json 2> $OUT/prof.err || { tail $OUT/prof.err; exit 1; }
python3 - <<'PY'
import csv, json
for r in csv.DictReader(open('gpurun_out/r3rp/prof/bench_kernel_stats.csv')):
    if any(k in r['Name'] for k in ('lean','locate','heavy')): print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1000,1), 'us')
d = json.load(open('gpurun_out/r3rp/c4_bench_under_rocprof.json'))
print('bench under rocprof', d['ms_per_step'], d['kernel_ms'], d['roofline']['kernel_ms'])
PY
