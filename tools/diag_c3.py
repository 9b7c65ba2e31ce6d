"""Diagnostics: where the C3 (coverageRnaRef) pileup time goes -- one plan per column part.

    python tools/diag_c3.py        (GPU box; RCP_LIB_PATH selects a library variant)
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import synthetic  # noqa: E402
from recoup_amd.engine import Bins, Plan, ReadSet  # noqa: E402


def timed(plan, out):
    for _ in range(2):
        plan.execute(out)
    plan.status()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    ts = []
    for _ in range(10):
        ev[0].record()
        plan.execute_stages(1, out)
        ev[1].record()
        plan.execute_stages(2, out)
        ev[2].record()
        plan.execute_stages(4, out)
        ev[3].record()
        torch.cuda.synchronize()
        ts.append([ev[i].elapsed_time(ev[i + 1]) for i in range(3)])
    return np.median(np.array(ts), axis=0)


def main():
    d = synthetic.c3(device="cuda:0")
    rows = synthetic.rna_rows(d)
    rs = ReadSet(*d["reads"], d["seqlen"], device=0)
    fb, cb, fl = d["flank_bins"], d["region_bins"], d["flank"]
    cases = [
        ("all parts", [("upstream", fb), ("center", cb), ("downstream", fb)]),
        ("upstream only", [("upstream", fb)]),
        ("center only", [("center", cb)]),
        ("downstream only", [("downstream", fb)]),
    ]
    only = sys.argv[1:]  # case names to run (default: all)
    for name, parts in cases:
        if only and name.split()[0] not in only:
            continue
        plan = Plan(rs, rows, Bins(parts, flank=fl), kernel=os.environ.get("DIAG_KERNEL", "auto"),
                    heavy_threshold=int(os.environ.get("DIAG_HEAVY", "-1")))
        out = plan.empty_output()
        t = timed(plan, out)
        plan.execute(out)
        info = {"heavy_rows": plan.heavy_rows()}
        info.update({k: plan.info[k] for k in ("n_cols", "n_interp_rows", "lds_bytes", "grid", "chunk_positions",
                                          "pileup_kernel")})
        print(f"{name:16s} locate {t[0]:.3f}  pileup {t[1]:.3f}  interp {t[2]:.3f} ms  {info}", flush=True)
        del plan, out


if __name__ == "__main__":
    main()
