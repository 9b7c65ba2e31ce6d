"""Calibration factors for FETCH_SIZE / WRITE_SIZE from tools/fetch_calib under rocprofv3 --pmc.

    python tools/pmc_calib.py OUT_DIR [OUT_JSON]

OUT_DIR/fetch/*counter_collection.csv (FETCH_SIZE) and OUT_DIR/write/... (WRITE_SIZE), both in
KiB per dispatch.  Each calibration kernel moves exactly 2 GiB per dispatch; the factor is
bytes / (counter x 1024), averaged over the dispatches of each kernel."""
import csv
import glob
import json
import os
import sys

BYTES = 2 << 30


def per_kernel(path, counter):
    acc = {}
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if row["Counter_Name"] != counter:
                continue
            name = row["Kernel_Name"].split("(")[0]
            acc.setdefault(name, []).append(float(row["Counter_Value"]) * 1024.0)
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main():
    d = sys.argv[1]
    fetch = per_kernel(os.path.join(d, "fetch"), "FETCH_SIZE")
    write = per_kernel(os.path.join(d, "write"), "WRITE_SIZE")
    res = {"bytes_per_dispatch": BYTES,
           "fetch_factor": {k: BYTES / v for k, v in fetch.items() if k.startswith("read") and v > 0},
           "write_factor": {k: BYTES / v for k, v in write.items() if k.startswith("write") and v > 0},
           "fetch_counter_bytes": fetch, "write_counter_bytes": write}
    txt = json.dumps(res, indent=1)
    print(txt)
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(txt + "\n")


if __name__ == "__main__":
    main()
