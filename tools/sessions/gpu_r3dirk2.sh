# inline-key directory: rocprof kernel averages per variant (C4 and C2, one pass in flight)
export TMPDIR=/tmp
OUT=gpurun_out/dirk2; mkdir -p $OUT
for c in c4 c2; do
  for v in base q2 q2w5 q4 base q2 q2w5 q4; do
    RCP_LIB_PATH=build_var/$v/librecoup_amd.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$v-$c -o p -- \
      python3 bench.py --config $c --no-cpu --no-e2e --inflight 1 --steps 30 > $OUT/$v-$c.json 2> $OUT/$v-$c.err || { tail $OUT/$v-$c.err; exit 1; }
    python3 - $OUT/$v-$c $v $c <<'PY' | tee -a $OUT/ab.log
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/p_kernel_stats.csv", recursive=True)[0]
row = {r["Name"].split("(")[0][:40]: float(r["AverageNs"]) / 1000 for r in csv.DictReader(open(f))}
print(sys.argv[2], sys.argv[3], {k: round(x, 1) for k, x in row.items() if "locate" in k or "lean" in k or "pileup" in k})
PY
  done
done
