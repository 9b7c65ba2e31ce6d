"""C4's reads in generation order (unsorted, as recoup_test_data's are) into a readset, in the
forms a host caller can hand them over, with RCP_TRACE=1 (staged copies and build phases):
  codes+ends   one chromosome code and one end per read (bench e2e any_order)
  codes+wruns  one code per read, widths as runs (r/R/rcp.R for unsorted reads of few widths)
  runs+wruns   seqnames as its Rle runs (unsorted: about one run per read) and width runs
    python tools/diag_unsorted.py [reps] [forms...]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import synthetic  # noqa: E402
from recoup_amd.engine import ReadSet  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
want = sys.argv[2:] or ["codes+ends", "codes+wruns", "runs+wruns"]
d = synthetic.c4(device="cuda:0")
chrom, start, end, strand = d["reads"]
w = (end - start + 1).to(torch.int32)
wv, wl = torch.unique_consecutive(w, return_counts=True)
wruns = (wv.cpu().numpy(), wl.to(torch.int64).cpu().numpy())
cv, cl = torch.unique_consecutive(chrom, return_counts=True)
cruns = (cv.to(torch.int32).cpu().numpy(), cl.to(torch.int64).cpu().numpy())
h = [x.cpu().numpy() for x in (chrom, start, end, strand)]
forms = {"codes+ends": h, "codes+wruns": [h[0], h[1], wruns, h[3]], "runs+wruns": [cruns, h[1], wruns, h[3]]}
print(f"{len(h[1])} reads, {len(cruns[0])} seqnames runs, {len(wruns[0])} width runs", file=sys.stderr)
ref = None
for name in want:
    for k in range(reps):
        os.environ["RCP_TRACE"] = "1" if k == reps - 1 else ""
        if not os.environ["RCP_TRACE"]:
            del os.environ["RCP_TRACE"]
        torch.cuda.synchronize()
        a = time.perf_counter()
        rs = ReadSet(*forms[name], d["seqlen"], device=0)
        torch.cuda.synchronize()
        print(f"{name} readset {k}: {(time.perf_counter() - a) * 1e3:.2f} ms", file=sys.stderr, flush=True)
        del rs
