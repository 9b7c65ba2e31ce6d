"""Diagnostics: pileup kernel time under workload variants (C4 shape)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import synthetic  # noqa: E402
from recoup_amd.engine import Bins, Plan, ReadSet, RowTable  # noqa: E402


def run(name, check_heavy=False, **kw):
    d = synthetic.c4(device="cuda:0", **kw)
    reg = d["regions"]
    rs = ReadSet(*d["reads"], d["seqlen"], device=0)
    rows = RowTable.from_ranges(reg["chrom"], reg["start"], reg["end"], reg["strand"])
    plan = Plan(rs, rows, Bins([("whole", d["n_bins"])]))
    out = plan.empty_output()
    for _ in range(2):
        plan.execute(out)
    plan.status()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    ts = []
    for _ in range(5):
        ev[0].record()
        plan.execute_stages(1, out)
        ev[1].record()
        plan.execute_stages(2, out)
        ev[2].record()
        plan.execute_stages(4, out)
        ev[3].record()
        torch.cuda.synchronize()
        ts.append([ev[i].elapsed_time(ev[i + 1]) for i in range(3)])
    ts = np.median(np.array(ts), axis=0)
    # pileup alone, back to back: 3 blocks of 20 launches, best block (less clock noise)
    blk = []
    for _ in range(3):
        ev[0].record()
        for _ in range(20):
            plan.execute_stages(2, out)
        ev[1].record()
        torch.cuda.synchronize()
        blk.append(ev[0].elapsed_time(ev[1]) / 20)
    ts[1] = min(blk)
    n_ovl = synthetic.n_overlaps(d["reads"], reg, d["width"]).astype(np.int64)
    byt = 8 * n_ovl.sum() + 16 * len(n_ovl) + 8 * len(n_ovl) * plan.n_cols
    print(f"{name:34s} locate+heavy {ts[0]:7.3f} ms  pileup {ts[1]:7.3f} ms ({byt / ts[1] / 1e6:7.1f} GB/s)  "
          f"n_ovl {n_ovl.sum():>10d} max {n_ovl.max():>8d}  lds {plan.info['lds_bytes']}", flush=True)
    if check_heavy:
        ref = out.clone()
        p2 = Plan(rs, rows, Bins([("whole", d["n_bins"])]), heavy_threshold=0)
        o2 = p2.execute()
        p2.status()
        print("   heavy path == plain path:", bool(torch.equal(ref, o2)), flush=True)
    del plan, rs, d


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "volume":
        run("c4 default (skewed, 92M ovl)")
        run("c4 no reads", n_reads=1000)
        run("c4 uniform 200M reads", enriched=0.0)
        run("c4 uniform 600M reads", enriched=0.0, n_reads=600_000_000)
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "quick":
        run("c4 default")
        run("c4 uniform reads only", enriched=0.0)
        sys.exit(0)
    run("c4 default", check_heavy=True)
    run("c4 uniform reads only", enriched=0.0)
    run("c4 no reads", n_reads=1000)
    run("c4 20M reads", n_reads=20_000_000)
