#!/bin/bash
# interpolation kernel ablations on C3: i1 no spline elimination chains, i2 no reads, i3 neither
OUT=gpurun_out/r3ia
mkdir -p $OUT
export TMPDIR=/tmp
for v in base i1 i2 i3; do
RCP_LIB_PATH=build_var/$v/librecoup_amd.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$v -o p -- \
  python3 bench.py --config c3 --no-cpu --no-e2e --steps 20 --inflight 1 > $OUT/$v.json 2> $OUT/$v.err || { tail $OUT/$v.err; exit 1; }
python3 -c "
import csv
for r in csv.DictReader(open('$OUT/$v/p_kernel_stats.csv')):
    if 'interp' in r['Name'] or 'rows_kernel' in r['Name']: print('$v', r['Name'][:40], r['Calls'], round(float(r['AverageNs'])/1000,1), 'us')
"
done
