#!/bin/bash
# Locate-kernel ablations (GPU box): rocprofv3 kernel stats of tools/diag_lean.py (C4) per
# library variant in build_var/<name>/.   tools/locate_abl.sh OUTDIR name1 name2 ...
set -e
OUT=$1; shift
export TMPDIR=/tmp
for v in "$@"; do
    RCP_LIB_PATH=build_var/$v/librecoup_amd.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
        -d "$OUT/$v" -o p -- python3 tools/diag_lean.py > "$OUT/$v.log" 2>&1
    python3 - "$OUT/$v" "$v" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/p_kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "rcp_" in r["Name"] and ("locate" in r["Name"] or "heavy" in r["Name"] or "lean" in r["Name"]):
            print(sys.argv[2], r["Name"][:40], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
done
