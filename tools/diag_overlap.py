"""Two passes in flight: C4 (or another config) with two plans of the same region table on one
readset (two samples' worth of passes), executed alternately on two HIP streams, vs the same
passes on one stream.  ms per pass, and the outputs checked equal.

    python tools/diag_overlap.py [c4|c5|c2] [steps]"""
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
rs = ReadSet(*d["reads"], d["seqlen"], device=0)
rows = RowTable.from_ranges(reg["chrom"], reg["start"], reg["end"], reg["strand"])
bins = Bins([("whole", d["n_bins"])]) if d["n_bins"] else Bins([("whole", 0, sum(d["flank"]))])
plans = [Plan(rs, rows, bins, out_ld="padded") for _ in range(2)]
outs = [p.empty_output() for p in plans]
streams = [torch.cuda.Stream(), torch.cuda.Stream()]


def run(two):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for k in range(K):
        i = k & 1
        plans[i].execute(outs[i], stream=streams[i] if two else streams[0])
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / K * 1e3


for _ in range(2):
    run(False)
    run(True)
res = {"one_stream_ms": [round(run(False), 4) for _ in range(3)], "two_streams_ms": [round(run(True), 4) for _ in range(3)]}
res["equal"] = bool(torch.equal(outs[0], outs[1]))
print(cfg, res, flush=True)
