"""One GPU's shard k/N of the C4 (or $CFG) workload (as bench.py --sim-shard builds it) on each pileup
kernel: ms per pass (D = 1, execute after execute), the stage times, and bit-equality with the
default plan.   python tools/diag_shard_kernels.py [K/N] [kernels...]   (kernel:C:H = min_col_chunks C, heavy_threshold H)"""
import os
import sys
import time
from types import SimpleNamespace

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from recoup_amd.engine import Plan, ReadSet  # noqa: E402

spec = sys.argv[1] if len(sys.argv) > 1 else "0/8"
kernels = sys.argv[2:] or ["auto", "rows", "general"]
k, n = (int(x) for x in spec.split("/"))
args = SimpleNamespace(config=os.environ.get("CFG", "c4"), seed=20261015, reads=None, regions=None)
data, rows_all, bins, ovl = bench.workload(args, "cuda:0")
lo, hi, _ = bench.shard_of(rows_all, ovl, n, k)
rows = bench.subset_rows(rows_all, lo, hi) if n > 1 else rows_all
reads = bench.reads_for_rows(data["reads"], rows, len(data["seqlen"])) if n > 1 else data["reads"]
rs = ReadSet(*reads, data["seqlen"], device=0)
ref = None
for kern in kernels:
    name, _, rest = kern.partition(":")
    mcc, _, heavy = rest.partition(":")
    plan = Plan(rs, rows, bins, kernel=name, out_ld="padded", min_col_chunks=int(mcc or 0),
                heavy_threshold=int(heavy or -1))
    out = plan.empty_output()
    for _ in range(5):
        plan.execute(out)
    plan.status()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(50):
        plan.execute(out)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t) / 50 * 1e3
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    st = [0.0, 0.0]
    for _ in range(20):
        ev[0].record()
        plan.execute_stages(1, out)
        ev[1].record()
        plan.execute_stages(2, out)
        ev[2].record()
        torch.cuda.synchronize()
        st[0] += ev[0].elapsed_time(ev[1]) / 20
        st[1] += ev[1].elapsed_time(ev[2]) / 20
    plan.status()
    m = out[:, :plan.n_rows].clone()
    same = None if ref is None else bool(torch.equal(m.view(torch.int64), ref.view(torch.int64)))
    if ref is None:
        ref = m
    print(f"{args.config} {spec} {kern:8s} kernel {plan.info['pileup_kernel']} fold {plan.info['fold']} grid {plan.info['grid']} ms/pass {ms:.4f} "
          f"locate {st[0]:.4f} pileup {st[1]:.4f} same_as_first {same}", flush=True)
