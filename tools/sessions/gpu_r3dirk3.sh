# inline-key directory adopted (14 keys): full GPU suite, rocprof locate C5 / C3 base vs q4, default bench
export TMPDIR=/tmp
OUT=gpurun_out/dirk3; mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1; st=$?; tail -3 $OUT/tests.log; [ $st -eq 0 ] || exit $st
for c in c5 c3; do
  for v in base q4 base q4; do
    RCP_LIB_PATH=build_var/$v/librecoup_amd.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$v-$c -o p -- \
      python3 bench.py --config $c --no-cpu --no-e2e --inflight 1 --steps 30 > $OUT/$v-$c.json 2> $OUT/$v-$c.err || { tail $OUT/$v-$c.err; exit 1; }
    python3 - $OUT/$v-$c $v $c <<'PY' | tee -a $OUT/ab.log
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/p_kernel_stats.csv", recursive=True)[0]
row = {r["Name"].split("(")[0][:40]: float(r["AverageNs"]) / 1000 for r in csv.DictReader(open(f))}
print(sys.argv[2], sys.argv[3], {k: round(x, 1) for k, x in sorted(row.items(), key=lambda kv: -kv[1])[:5]})
PY
  done
done
timeout -k 10 600 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err; st=$?; cat $OUT/bench_default.json; exit $st
