"""Per-kernel averages of rocprofv3 --pmc counter_collection.csv files (KiB counters x 1024).

    python tools/pmc_kernels.py PMC_DIR [name-substring ...]
"""
import csv
import glob
import os
import sys
from collections import defaultdict

d = sys.argv[1]
keys = sys.argv[2:]
acc = defaultdict(list)
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        name = row["Kernel_Name"]
        if keys and not any(k in name for k in keys):
            continue
        acc[(name[:80], row["Counter_Name"])].append(float(row["Counter_Value"]))
for (name, ctr), v in sorted(acc.items()):
    scale = 1024.0 if ctr in ("FETCH_SIZE", "WRITE_SIZE") else 1.0
    print(f"{name:80s} {ctr:12s} n={len(v):3d} avg={sum(v) / len(v) * scale:.4g}")
