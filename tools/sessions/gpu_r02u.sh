#!/bin/bash
# rocprof kernel stats with one pass in flight (durations not overlapped), N=2 rehearsal on one GPU
OUT=gpurun_out/r02u
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c4 -o bench -- \
    python3 bench.py --no-cpu --no-e2e --inflight 1 --traffic profiles/traffic_c4.json > $OUT/c4_bench_under_rocprof.json 2> $OUT/prof_c4.err || { tail $OUT/prof_c4.err; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c3 -o bench -- \
    python3 bench.py --config c3 --no-cpu --no-e2e --inflight 1 > $OUT/c3_bench_under_rocprof.json 2> $OUT/prof_c3.err || { tail $OUT/prof_c3.err; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_s08 -o bench -- \
    python3 bench.py --no-cpu --no-e2e --inflight 1 --sim-shard 0/8 > $OUT/s08_bench_under_rocprof.json 2> $OUT/prof_s08.err || { tail $OUT/prof_s08.err; exit 1; }
RCP_SHARE_GPU=1 RCP_DIST_BACKEND=gloo timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --no-cpu --verify-gather \
    > $OUT/c4_n2_rehearsal.json 2> $OUT/c4_n2_rehearsal.err || { tail $OUT/c4_n2_rehearsal.err; exit 1; }
cat $OUT/c4_n2_rehearsal.json
find $OUT -name "*kernel_stats.csv" | while read f; do echo "== $f"; python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    if 'rcp_' in r['Name']: print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,2), 'us')
"; done
for f in $OUT/*under_rocprof.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', round(d['ms_per_step'],4), d['kernel_ms'])"; done
