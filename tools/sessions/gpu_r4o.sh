#!/bin/bash
# round 4: same-box A/B of the round-3 final tree (build_var/r03) and this tree, kernel times by
# rocprofv3 on C4 and C2 (tools/prof_c4.py), alternating
OUT=gpurun_out/r4o
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
  for t in r03 new; do
    dir=build_var/r03
    [ $t = new ] && dir=.
    for c in c4; do
      (cd $dir && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/${t}_${c}_$rep -o p -- python3 tools/prof_c4.py $c > $GRAFT_REPO_ROOT/$OUT/${t}_${c}_$rep.log 2>&1) || { tail $OUT/${t}_${c}_$rep.log; exit 1; }
      python3 - $OUT/${t}_${c}_$rep/p_kernel_stats.csv $t $c <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r['Name']
    if any(k in n for k in ('locate', 'heavy_pileup', 'pileup_lean', 'pileup_bins', 'pileup_kernel')):
        print(sys.argv[2], sys.argv[3], n[:50], r['Calls'], round(float(r['AverageNs']) / 1000, 2), 'us')
PY
    done
  done
done
