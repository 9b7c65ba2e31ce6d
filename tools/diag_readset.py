"""Readset creation from host arrays, repeated (variance of the C5-sized H2D + layouts).

    python tools/diag_readset.py [c5|c4] [reps]     (RCP_TRACE=1: per-phase lines of each build;
                                                     STRANDED=1: the strand-split layout as well)"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import synthetic  # noqa: E402
from recoup_amd.engine import ReadSet  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c5"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 6
d = getattr(synthetic, cfg)(device="cuda:0")
host = [x.cpu().numpy() for x in d["reads"]]
print("free/total GB", [round(x / 2**30, 1) for x in torch.cuda.mem_get_info()], flush=True)
for k in range(reps):
    torch.cuda.synchronize()
    a = time.perf_counter()
    rs = ReadSet(*host, d["seqlen"], device=0)
    if os.environ.get("STRANDED"):
        rs.stream_off  # builds the strand-split layout too
    torch.cuda.synchronize()
    b = time.perf_counter()
    del rs
    torch.cuda.synchronize()
    c = time.perf_counter()
    free = torch.cuda.mem_get_info()[0] / 2**30
    print(f"rep {k}: create {(b - a) * 1e3:.1f} ms, destroy {(c - b) * 1e3:.1f} ms, free {free:.1f} GB", flush=True)
