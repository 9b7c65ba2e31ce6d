"""Where the host-to-host time of the C ABI one-shot path goes (C4 by default).

    python tools/diag_e2e.py [c4|c2|c5]

Times, each a few times: rcp_readset_create from host arrays vs from device arrays (the
difference is the H2D of the reads), rcp_plan_create, rcp_plan_execute, and rcp_profile
(plan + execute + D2H into a touched host matrix)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import synthetic  # noqa: E402
from recoup_amd.engine import Bins, Plan, ReadSet, RowTable, profile_host  # noqa: E402


def t(fn, reps=3):
    out = []
    for _ in range(reps):
        torch.cuda.synchronize()
        a = time.perf_counter()
        r = fn()
        torch.cuda.synchronize()
        out.append((time.perf_counter() - a) * 1e3)
        del r
    return out


cfg = sys.argv[1] if len(sys.argv) > 1 else "c4"
d = getattr(synthetic, cfg)(device="cuda:0")
reg = d["regions"]
rows = RowTable.from_ranges(reg["chrom"], reg["start"], reg["end"], reg["strand"])
bins = Bins([("whole", d["n_bins"])]) if d["n_bins"] else Bins([("whole", 0, sum(d["flank"]))])
host = [x.cpu().numpy() for x in d["reads"]]
res = {}
res["readset_from_device_ms"] = t(lambda: ReadSet(*d["reads"], d["seqlen"], device=0))
res["readset_from_host_ms"] = t(lambda: ReadSet(*host, d["seqlen"], device=0))
rs = ReadSet(*d["reads"], d["seqlen"], device=0)
res["plan_create_ms"] = t(lambda: Plan(rs, rows, bins))
plan = Plan(rs, rows, bins)
o = plan.empty_output()
res["execute_ms"] = t(lambda: plan.execute(o), reps=5)
out = np.zeros((bins.n_cols, rows.n_rows))
res["profile_one_shot_ms"] = t(lambda: profile_host(rs, rows, bins, out))
res["d2h_torch_pageable_ms"] = t(lambda: o.cpu())
ref = o.cpu().numpy()
profile_host(rs, rows, bins, out)
res["one_shot_matches_device"] = bool(np.array_equal(out.view(np.uint64), ref.view(np.uint64)))
print({k: ([round(x, 2) for x in v] if isinstance(v, list) else v) for k, v in res.items()}, flush=True)
