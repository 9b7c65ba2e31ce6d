#!/bin/bash
OUT=gpurun_out/r3z2
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o p -- python3 bench.py --config c3 --no-cpu --no-e2e --inflight 1 > $OUT/c3.json 2> $OUT/c3.err || { tail $OUT/c3.err; exit 1; }
grep -E "interp|rows|locate|heavy" $OUT/prof/p_kernel_stats.csv | cut -d, -f1,2,4
python3 - <<'PY'
import csv
rows=[r for r in csv.DictReader(open('gpurun_out/r3z2/prof/p_kernel_trace.csv')) if 'interp_kernel' in r['Kernel_Name']]
r=rows[-1]
print({k: r[k] for k in ('LDS_Block_Size','Scratch_Size','VGPR_Count','SGPR_Count','Workgroup_Size_X','Grid_Size_X')})
PY
