#!/bin/bash
# round 4 end: smoke, the measurement set (tools/round_profile.sh: C4 PMC traffic, C4 bench +
# rocprofv3 kernel summary, C2 / C3 / C5 lines), 1/8-shard rehearsals (C4, C5)
OUT=gpurun_out/${R4K_OUT:-r4k}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -30 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 1000 bash tools/round_profile.sh $OUT/round > $OUT/round.log 2>&1 || { tail -30 $OUT/round.log; exit 1; }
grep -h '"metric"' $OUT/round/*_bench.json | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['config']['workload'][:3], d['value'], d['ms_per_step'], d.get('single_pass_ms'), d['roofline']['frac'] if d.get('roofline') else None)"
for spec in c4:0/8 c5:0/8; do
  timeout -k 10 400 python3 bench.py --config ${spec%%:*} --sim-shard ${spec#*:} --no-cpu --no-e2e > $OUT/shard_${spec%%:*}.json 2> $OUT/shard_${spec%%:*}.err || { tail $OUT/shard_${spec%%:*}.err; exit 1; }
  cat $OUT/shard_${spec%%:*}.json
done
for c in c4 c5; do
  CFG=$c timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_shard_$c -o p -- python3 tools/diag_shard_kernels.py 0/8 auto > $OUT/prof_shard_$c.log 2>&1 || { tail $OUT/prof_shard_$c.log; exit 1; }
  python3 - $OUT/prof_shard_$c/p_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'rcp_' in r['Name']:
        print(r['Name'][:60], r['Calls'], round(float(r['AverageNs']) / 1000, 2), 'us')
PY
done
STRANDED=1 timeout -k 10 300 python3 tools/diag_readset.py c4 8 > $OUT/readset_c4.log 2>&1 || { tail $OUT/readset_c4.log; exit 1; }
grep rep $OUT/readset_c4.log
