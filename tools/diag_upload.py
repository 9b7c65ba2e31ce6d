"""C4's reads as a sorted BAM gives them (seqnames and widths as runs) into a readset, repeated,
with RCP_TRACE=1: the staged copies' lines ([stage] h2d / h2d-packed) and the build phases."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import synthetic  # noqa: E402
from recoup_amd.engine import ReadSet  # noqa: E402

d = synthetic.c4(device="cuda:0")
chrom, start, end, strand = d["reads"]
order = torch.argsort((chrom.to(torch.int64) << 32) | start.to(torch.int64))
sc = chrom[order]
rv, rl = torch.unique_consecutive(sc, return_counts=True)
w = (end[order] - start[order] + 1).to(torch.int32)
wv, wl = torch.unique_consecutive(w, return_counts=True)
host = [(rv.to(torch.int32).cpu().numpy(), rl.to(torch.int64).cpu().numpy()), start[order].cpu().numpy(),
        (wv.cpu().numpy(), wl.to(torch.int64).cpu().numpy()), strand[order].cpu().numpy()]
del order, sc, w
os.environ["RCP_TRACE"] = "1"
for k in range(4):
    torch.cuda.synchronize()
    a = time.perf_counter()
    rs = ReadSet(*host, d["seqlen"], device=0)
    print(f"readset {k}: {(time.perf_counter() - a) * 1e3:.2f} ms", file=sys.stderr, flush=True)
    del rs
