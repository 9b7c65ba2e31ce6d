"""HBM traffic per launch of the pileup kernel from rocprofv3 --pmc passes (tools/pmc.sh).

    python tools/pmc_traffic.py PMC_DIR [OUT_JSON]

Reads PMC_DIR/fetch/*_counter_collection.csv (FETCH_SIZE) and PMC_DIR/write/... (WRITE_SIZE),
both in KiB per dispatch, averages over the pileup kernel's dispatches (lean or general) and applies the gfx950
correction of MI355X_MICROARCH.md (HBM section): FETCH_SIZE reports half the bytes of wide
coalesced reads, so it is doubled; WRITE_SIZE is exact for 16-B-per-lane streaming stores.
PMC_DIR/meta.json (written by tools/prof_c4.py via PROF_META) names the workload so bench.py
only attaches the number to the same configuration.
"""
import csv
import glob
import json
import os
import sys

KERNELS = ("rcp_pileup_lean_kernel<", "rcp_pileup_kernel<")  # whichever the plan launched


def per_launch(path, counter):
    for kernel in KERNELS:
        vals = []
        for f in glob.glob(os.path.join(path, "*counter_collection.csv")):
            for row in csv.DictReader(open(f)):
                if kernel in row["Kernel_Name"] and row["Counter_Name"] == counter:
                    vals.append(float(row["Counter_Value"]) * 1024.0)
        if vals:
            return sum(vals) / len(vals), len(vals), kernel.rstrip("<")
    raise SystemExit(f"no {counter} rows for {KERNELS} under {path}")


def main():
    d = sys.argv[1]
    out = sys.argv[2] if len(sys.argv) > 2 else None
    fetch, nf, kernel = per_launch(os.path.join(d, "fetch"), "FETCH_SIZE")
    write, nw, _ = per_launch(os.path.join(d, "write"), "WRITE_SIZE")
    meta = json.load(open(os.path.join(d, "meta.json")))
    res = dict(meta)
    res.update({"kernel": kernel, "fetch_size_bytes_raw": fetch, "fetch_bytes": 2 * fetch,
                "write_bytes": write, "hbm_bytes_per_launch": 2 * fetch + write, "dispatches": [nf, nw],
                "correction": "FETCH_SIZE x2 (gfx950 wide-read tally), WRITE_SIZE as is"})
    txt = json.dumps(res, indent=1)
    print(txt)
    if out:
        open(out, "w").write(txt + "\n")


if __name__ == "__main__":
    main()
