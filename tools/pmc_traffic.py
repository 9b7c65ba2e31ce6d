"""HBM traffic per launch of the pileup kernel from rocprofv3 --pmc passes (tools/pmc.sh).

    python tools/pmc_traffic.py PMC_DIR [OUT_JSON] [CALIB_JSON]

Reads PMC_DIR/fetch/*_counter_collection.csv (FETCH_SIZE) and PMC_DIR/write/... (WRITE_SIZE),
both in KiB per dispatch, averages over the pileup kernel's dispatches (lean or general) and applies the gfx950
correction: MI355X_MICROARCH.md (HBM section) documents FETCH_SIZE = 1/2 of the bytes for
16-B-per-lane coalesced reads; the pileup streams 8-B int2 reads (4-B starts over a
uniform-width readset), so the factor measured for that shape by tools/fetch_calib.hip
(CALIB_JSON from tools/pmc_calib.py, kernel read8_plain / read4_plain) is used when given, else x2.  WRITE_SIZE: the calibrated factor of the 8-B non-temporal
column-segment stores (write8_seg16), else as is.
PMC_DIR/meta.json (written by tools/prof_c4.py via PROF_META) names the workload so bench.py
only attaches the number to the same configuration.
"""
import csv
import glob
import json
import os
import sys

KERNELS = ("rcp_pileup_lean_kernel<", "rcp_pileup_kernel<", "rcp_pileup_rows_kernel<", "rcp_pileup_bins_kernel<")  # whichever the plan launched


def per_launch(path, counter):
    for kernel in KERNELS:
        vals, names = [], set()
        for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
            for row in csv.DictReader(open(f)):
                if kernel in row["Kernel_Name"] and row["Counter_Name"] == counter:
                    vals.append(float(row["Counter_Value"]) * 1024.0)
                    names.add(row["Kernel_Name"])
        if vals:
            return sum(vals) / len(vals), len(vals), kernel.rstrip("<("), names
    raise SystemExit(f"no {counter} rows for {KERNELS} under {path}")


def main():
    d = sys.argv[1]
    out = sys.argv[2] if len(sys.argv) > 2 else None
    fetch, nf, kernel, names = per_launch(os.path.join(d, "fetch"), "FETCH_SIZE")
    write, nw, _, _ = per_launch(os.path.join(d, "write"), "WRITE_SIZE")
    # the lean kernel over a uniform-width readset (last template argument true) streams 4-B starts
    starts_only = any(n.startswith("void rcp_pileup_lean_kernel<") and ", true>(" in n for n in names)
    shape, key = ("4-B/lane int32 starts", "read4_plain") if starts_only else ("8-B/lane int2 reads", "read8_plain")
    fk, wk, how = 2.0, 1.0, f"FETCH_SIZE x2 (guide's 16-B/lane rule; the kernel streams {shape}), WRITE_SIZE as is"
    if len(sys.argv) > 3:
        cal = json.load(open(sys.argv[3]))
        if key in cal["fetch_factor"]:
            fk = cal["fetch_factor"][key]
            how = f"FETCH_SIZE x{fk:.3f} (calibrated: {shape}, tools/fetch_calib.hip {key})"
        else:
            how = f"FETCH_SIZE x2 (no {key} calibration; the kernel streams {shape})"
        wk = cal["write_factor"].get("write8_seg16", 1.0)
        how += f", WRITE_SIZE x{wk:.3f} (calibrated: 8-B nt column-segment stores)"
    meta = json.load(open(os.path.join(d, "meta.json")))
    res = dict(meta)
    res.update({"kernel": kernel, "fetch_size_bytes_raw": fetch, "fetch_bytes": fk * fetch,
                "write_size_bytes_raw": write, "write_bytes": wk * write,
                "hbm_bytes_per_launch": fk * fetch + wk * write, "dispatches": [nf, nw], "correction": how})
    txt = json.dumps(res, indent=1)
    print(txt)
    if out:
        open(out, "w").write(txt + "\n")


if __name__ == "__main__":
    main()
