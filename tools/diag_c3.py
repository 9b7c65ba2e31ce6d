"""Find rows where the C3 profile differs from the oracle (diagnostic)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import synthetic  # noqa: E402
import oracle_rows  # noqa: E402
from recoup_amd.engine import Bins, Plan, ReadSet, RowTable  # noqa: E402

n_genes = int(sys.argv[1]) if len(sys.argv) > 1 else 25000
n_pairs = int(sys.argv[2]) if len(sys.argv) > 2 else 50_000_000
m = int(sys.argv[3]) if len(sys.argv) > 3 else 1500
d = synthetic.c3(device="cuda:0", n_genes=n_genes, n_pairs=n_pairs)
rows = synthetic.rna_rows(d)
bins = Bins([("upstream", 50), ("center", 500), ("downstream", 50)], flank=d["flank"])
rs = ReadSet(*d["reads"], d["seqlen"], device=0)
plan = Plan(rs, rows, bins)
print("info", plan.info, flush=True)
mat, valid = plan.run()
reads = tuple(t.cpu().numpy() for t in d["reads"])
ix = oracle_rows.index_for(reads, d["seqlen"])
sub = RowTable(rows.seg_off[:m + 1], rows.chrom[:rows.seg_off[m]], rows.start[:rows.seg_off[m]],
               rows.end[:rows.seg_off[m]], rows.strand[:rows.seg_off[m]], seg_group=rows.seg_group[:rows.seg_off[m]],
               group_is_list=rows.group_is_list)
cov = oracle_rows.row_coverage(ix, sub)
exp, ev = oracle_rows.profile(cov, bins)
print("valid equal:", np.array_equal(valid[:m], ev), "valid rows", ev.sum())
bad = ~np.isclose(mat[:m], exp, rtol=1e-9, atol=1e-12)
rb = np.nonzero(bad.any(axis=1))[0]
print("rows differing:", len(rb))
lens = np.array([len(c) if c is not None else -1 for c in cov])
nseg = np.diff(rows.seg_off[:m + 1])
for r in rb[:10]:
    cols = np.nonzero(bad[r])[0]
    print(f"row {r} len {lens[r]} nseg {nseg[r]} cols {cols[:8]}..({len(cols)}) gpu {mat[r, cols[:3]]} exp {exp[r, cols[:3]]}")
