#!/bin/bash
# Same-box A/B of library variants by rocprof kernel averages: tools/rocprof_ab.sh OUTDIR "cfgs" v1 v2 ...
#   (bench.py --inflight 1 under rocprofv3 --kernel-trace --stats; per run: ms per pass and the
#   average of every kernel launched more than 20 times; extra bench arguments in $BENCH_ARGS)
export TMPDIR=/tmp
OUT=$1; CFGS=$2; shift 2
mkdir -p $OUT
for c in $CFGS; do
  for v in "$@"; do
    RCP_LIB_PATH=build_var/$v/librecoup_amd.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$v-$c -o p -- \
      python3 bench.py --config $c --no-cpu --no-e2e --inflight 1 --steps 30 $BENCH_ARGS > $OUT/$v-$c.json 2> $OUT/$v-$c.err || { tail $OUT/$v-$c.err; exit 1; }
    python3 - $OUT/$v-$c $v $c $OUT/$v-$c.json <<'PY' | tee -a $OUT/ab.log
import csv, glob, json, sys
f = sorted(glob.glob(sys.argv[1] + "/**/p_kernel_stats.csv", recursive=True))[0]
row = {r["Name"].split("(")[0].replace("void ", "")[:34]: (float(r["AverageNs"]) / 1000, int(r["Calls"])) for r in csv.DictReader(open(f))}
ms = json.load(open(sys.argv[4]))["ms_per_step"]
print(sys.argv[2], sys.argv[3], round(ms, 4), {k: round(x[0], 1) for k, x in row.items() if x[1] > 20 and "rocclr" not in k})
PY
  done
done
