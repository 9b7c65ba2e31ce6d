"""Per-dispatch averages of rocprofv3 counter CSVs: tools/pmc_sum.py [-k PATTERN] DIR..."""
import collections
import csv
import glob
import sys

# -k PATTERN: kernels whose name contains PATTERN (default "pileup")
args = sys.argv[1:]
pat = "pileup"
if args[:1] == ["-k"]:
    pat, args = args[1], args[2:]
for d in args:
    for f in sorted(glob.glob(f"{d}/*/p_counter_collection.csv")):
        rows = list(csv.DictReader(open(f)))
        agg = collections.defaultdict(lambda: collections.defaultdict(float))
        disp = collections.defaultdict(set)
        for r in rows:
            k = r["Kernel_Name"].split("(")[0][:48]
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add(r["Dispatch_Id"])
        for k, v in agg.items():
            if pat in k:
                n = len(disp[k])
                print(f"{f.split('/')[-2]:5s} {k:48s}", " ".join(f"{c}={x / n:.4g}" for c, x in sorted(v.items())))
