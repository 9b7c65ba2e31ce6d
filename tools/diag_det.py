"""Determinism / isolation check of one config's pass: the same plan twice, a second plan of the
same workload, and two plans on two streams concurrently -- outputs compared on the valid rows.

    python tools/diag_det.py [c3|c4|c5|c2]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import synthetic  # noqa: E402
from recoup_amd.engine import Bins, Plan, ReadSet, RowTable  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
d = getattr(synthetic, cfg)(device="cuda:0")
if cfg == "c3":
    rows = synthetic.rna_rows(d)
    bins = Bins([("upstream", d["flank_bins"]), ("center", d["region_bins"]), ("downstream", d["flank_bins"])],
                flank=d["flank"])
else:
    reg = d["regions"]
    rows = RowTable.from_ranges(reg["chrom"], reg["start"], reg["end"], reg["strand"])
    bins = Bins([("whole", d["n_bins"])]) if d["n_bins"] else Bins([("whole", 0, sum(d["flank"]))])
rs = ReadSet(*d["reads"], d["seqlen"], device=0)
R = rows.n_rows
p1 = Plan(rs, rows, bins, out_ld="padded")
p2 = Plan(rs, rows, bins, out_ld="padded")
print("info", p1.info, flush=True)


def diff(a, b, what):
    a, b = a[:, :R], b[:, :R]
    ne = (a.view(torch.int64) != b.view(torch.int64))
    n = int(ne.sum())
    msg = f"{what}: {n} differing cells"
    if n:
        cols = torch.nonzero(ne.any(dim=1)).flatten().cpu().numpy()
        rws = torch.nonzero(ne.any(dim=0)).flatten().cpu().numpy()
        msg += f" in {len(cols)} cols ({cols[:8]}...) {len(rws)} rows ({rws[:8]}...); max |d| {float((a - b).abs().max()):.3g}"
    print(msg, flush=True)


o1 = p1.execute()
torch.cuda.synchronize()
o1b = p1.execute()
torch.cuda.synchronize()
diff(o1, o1b, "same plan twice")
o2 = p2.execute()
torch.cuda.synchronize()
diff(o1, o2, "second plan, sequential")
s = [torch.cuda.Stream(), torch.cuda.Stream()]
for k in range(6):
    (p1 if k % 2 == 0 else p2).execute(o1 if k % 2 == 0 else o2, stream=s[k % 2])
torch.cuda.synchronize()
diff(o1, o2, "two streams")
ref = p1.execute()
torch.cuda.synchronize()
diff(ref, o1, "after concurrency vs fresh")
# stress: many passes of one plan on one stream, each compared with the first
N = int(sys.argv[2]) if len(sys.argv) > 2 else 60
bad = 0
for k in range(N):
    o = p1.execute(o1)
    torch.cuda.synchronize()
    if not torch.equal(o[:, :R], ref[:, :R]):
        bad += 1
        if bad <= 3:
            diff(ref, o, f"one stream pass {k}")
print(f"one stream: {bad} of {N} passes differ", flush=True)
bad = 0
for k in range(N):
    (p1 if k % 2 == 0 else p2).execute(o1 if k % 2 == 0 else o2, stream=s[k % 2])
    if k % 2 == 1:
        torch.cuda.synchronize()
        for o, w in ((o1, "p1"), (o2, "p2")):
            if not torch.equal(o[:, :R], ref[:, :R]):
                bad += 1
                if bad <= 3:
                    diff(ref, o, f"two streams pass {k} {w}")
print(f"two streams: {bad} of {N} pass results differ", flush=True)
