"""The R production path of one BASELINE config (c4 default; c2, c3, c5) for rocprofv3: readset,
rcp_coverage_rle (GPU pileup + RLE, runs to the host), rcp_profile_rle of those host runs --
ITERS times.  Prints per-phase wall times and the run count; checks the matrix bit-equal to
the fused pass once."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import synthetic  # noqa: E402
from recoup_amd.engine import Bins, Plan, ReadSet, RowTable, coverage_rle_host, profile_rle_arrays  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c4"
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
ref, _ = Plan(rs, rows, bins).run()
out = np.zeros((rows.n_rows, bins.n_cols), order="F")
for it in range(int(os.environ.get("ITERS", "3"))):
    tm = {}
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run_off, values, lengths, valid = coverage_rle_host(rs, rows, timing=tm)
    t1 = time.perf_counter()
    profile_rle_arrays(run_off, lengths, values, (valid == 0).astype(np.uint8), bins, 0, out)
    t2 = time.perf_counter()
    print(f"iter {it}: coverage_rle {1e3 * (t1 - t0):.1f} ms ({tm}), profile_rle {1e3 * (t2 - t1):.1f} ms, "
          f"{int(run_off[-1])} runs", flush=True)
    del run_off, values, lengths, valid  # (freed outside the timed calls)
print("equal_fused", bool(np.array_equal(out.view(np.int64), np.asfortranarray(ref).view(np.int64))))
