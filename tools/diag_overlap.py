"""Two passes in flight: C4 (or another config) with two plans of the same region table on one
readset (two samples' worth of passes), executed alternately on two HIP streams, vs the same
passes on one stream.  ms per pass, and the outputs checked equal.

    python tools/diag_overlap.py [c4|c5|c2] [steps] [K/N]   (K/N: rank K's shard of an N-way split)"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import synthetic  # noqa: E402
from recoup_amd.engine import Bins, Plan, ReadSet, RowTable  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c4"
K = int(sys.argv[2]) if len(sys.argv) > 2 else 20
d = getattr(synthetic, cfg)(device="cuda:0")
reg = d["regions"]
rows = RowTable.from_ranges(reg["chrom"], reg["start"], reg["end"], reg["strand"])
reads = d["reads"]
if len(sys.argv) > 3:
    import bench
    k, n = (int(x) for x in sys.argv[3].split("/"))
    ovl = synthetic.n_overlaps(d["reads"], reg, d["width"], device="cuda:0")
    lo, hi, _ = bench.shard_of(rows, ovl, n, k)
    rows = bench.subset_rows(rows, lo, hi)
    reads = bench.reads_for_rows(d["reads"], rows, len(d["seqlen"]))
rs = ReadSet(*reads, d["seqlen"], device=0)
bins = Bins([("whole", d["n_bins"])]) if d["n_bins"] else Bins([("whole", 0, sum(d["flank"]))])
plans = [Plan(rs, rows, bins, out_ld="padded") for _ in range(2)]
outs = [p.empty_output() for p in plans]
streams = [torch.cuda.Stream(), torch.cuda.Stream()]


def run(mode):
    """one: both plans on one stream; two: each plan on its stream (passes overlap freely);
    pipe: each plan on its stream, but a pass's pileup waits for the previous pass's pileup
    (only locate / heavy of pass k overlap pass k-1's pileup)."""
    torch.cuda.synchronize()
    t = time.perf_counter()
    prev = None
    for k in range(K):
        i = k & 1
        st = streams[i] if mode != "one" else streams[0]
        if mode == "pipe":
            plans[i].execute_stages(1, outs[i], stream=st)
            if prev is not None:
                st.wait_event(prev)
            plans[i].execute_stages(6, outs[i], stream=st)
            prev = torch.cuda.Event()
            prev.record(st)
        else:
            plans[i].execute(outs[i], stream=st)
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / K * 1e3


for _ in range(2):
    for m in ("one", "two", "pipe"):
        run(m)
res = {m: [round(run(m), 4) for _ in range(3)] for m in ("one", "two", "pipe")}
n = rows.n_rows
res["equal"] = bool(torch.equal(outs[0][:, :n], outs[1][:, :n]))
print(cfg, sys.argv[3] if len(sys.argv) > 3 else "", res, flush=True)
