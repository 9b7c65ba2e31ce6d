#!/bin/bash
# round 4: counters for the verdict items -- C2 bins-kernel instruction mix (SQ), C4 coverage
# (Rle) kernels' HBM traffic (FETCH_SIZE / WRITE_SIZE, separate passes)
OUT=gpurun_out/r4t
mkdir -p $OUT
export TMPDIR=/tmp
PASSES=sq timeout -k 10 400 bash tools/pmc.sh $OUT/pmc_c2 c2 || { tail $OUT/pmc_c2/*.log; exit 1; }
python3 tools/pmc_sum.py -k pileup $OUT/pmc_c2 | tee $OUT/c2_sq.txt
for c in FETCH_SIZE WRITE_SIZE; do
  ITERS=1 timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $OUT/rle_$c -o p -- python3 tools/prof_rle.py c4 > $OUT/rle_$c.log 2>&1 || { tail $OUT/rle_$c.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    agg = collections.defaultdict(list)
    for f in glob.glob(f"gpurun_out/r4t/rle_{c}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            n = r["Kernel_Name"]
            if any(k in n for k in ("pileup_kernel", "cov_runs", "rle_tile", "locate", "heavy")):
                agg[n.split("(")[0][:60]].append(float(r["Counter_Value"]) * 1024)
    for k, v in agg.items():
        print(c, k, len(v), "%.3f GB raw per dispatch" % (sum(v) / len(v) / 1e9))
PY
