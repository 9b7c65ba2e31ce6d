"""Minimal run of one BASELINE config (c4 default; c2, c3, c5) for rocprofv3 counter passes (one plan, a few
executes).  C3_PART=center keeps one column part of C3; SHARD=k/N one GPU's region shard (not C3)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import synthetic  # noqa: E402
from recoup_amd.engine import Bins, Plan, ReadSet, RowTable  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c4"
d = getattr(synthetic, cfg)(device="cuda:0")
rs = ReadSet(*d["reads"], d["seqlen"], device=0)
if cfg == "c3":  # coverageRnaRef rows, flank / centre / flank parts (as bench.py)
    rows = synthetic.rna_rows(d)
    parts = [("upstream", d["flank_bins"]), ("center", d["region_bins"]), ("downstream", d["flank_bins"])]
    if os.environ.get("C3_PART"):
        parts = [p for p in parts if p[0] == os.environ["C3_PART"]]
    bins = Bins(parts, flank=d["flank"])
    reg = {"start": rows.seg_off[1:]}
else:
    reg = d["regions"]
    rows = RowTable.from_ranges(reg["chrom"], reg["start"], reg["end"], reg["strand"])
    bins = Bins([("whole", d["n_bins"])]) if d["n_bins"] else Bins([("whole", 0, sum(d["flank"]))])
if os.environ.get("SHARD"):  # one GPU's shard k/N, as bench.py --sim-shard builds it
    import bench  # noqa: E402
    import numpy as np  # noqa: E402
    k, n = (int(x) for x in os.environ["SHARD"].split("/"))
    ovl = synthetic.n_overlaps(d["reads"], reg, d["width"], device="cuda:0").astype(np.int64)
    lo, hi, _ = bench.shard_of(rows, ovl, n, k)
    rows = bench.subset_rows(rows, lo, hi)
    rs = ReadSet(*bench.reads_for_rows(d["reads"], rows, len(d["seqlen"])), d["seqlen"], device=0)
plan = Plan(rs, rows, bins, out_ld="padded")  # as bench.py
out = plan.empty_output()
for _ in range(int(os.environ.get("ITERS", "3"))):
    plan.execute(out)
plan.status()
torch.cuda.synchronize()
print("ok", plan.info)
meta = os.environ.get("PROF_META")
if meta:
    import json
    with open(meta, "w") as f:
        json.dump({"config": cfg, "regions": len(reg["start"]), "reads": int(d["reads"][1].numel())}, f)
