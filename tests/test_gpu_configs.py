"""Every BASELINE.json configuration under -m gpu (the bench's workloads, synthetic.py):

  C2  full size: 10k TSS +-2 kb, 200 bins, 10M reads                  vs the CPU oracle
  C4  reduced:   20k peaks, 20M reads, Pareto hot peaks (heavy path)    vs the CPU oracle
  C4  full size: 200k peaks x 1000 bins, 200M reads                     size-independent properties
  C5  reduced:   2.5k regions x 4000 bp per base, 50M reads             vs the CPU oracle
  C3  reduced:   2.5k genes (exon lists + flanks), 5M read pairs         vs the CPU oracle

Integer numerators and per-base depth are bit-exact (means compared at rtol 1e-12; the
north_star bar is 1e-6); spline / neighborhood rows of C3 within rtol 1e-9.  The full C4
check uses SURVEY.md Appendix C's closed form: the depth summed over a region,
C(e) - C(s - 1) with C(x) = cnt_s(x)(x + 1) - sum(start <= x) - [cnt_e(< x) x - sum(end < x)],
computed with sorted keys and int64 prefix sums on the GPU, must equal 2 x the sum of the
row's 2-bp bin means, every 2 x mean must be an integer, and a row is valid iff a read
overlaps it."""
import os

import numpy as np
import pytest
import torch

import synthetic
from oracle import oracle as o
from recoup_amd.engine import Bins, Plan, ReadSet, RowTable

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def threads():
    try:
        return max(1, min(16, len(os.sched_getaffinity(0))))
    except AttributeError:
        return 4


def host_index(reads, seqlen):
    """The oracle's read index from device reads, handed over in (chrom, start) order."""
    c, s, e, st = reads
    order = torch.argsort((c.to(torch.int64) << 32) | s.to(torch.int64))
    h = [x[order].cpu().numpy() for x in (c, s, e, st)]
    return o.Index(*h, seqlen)


def single_rows(reg):
    return RowTable.from_ranges(reg["chrom"], reg["start"], reg["end"], reg["strand"])


def run(reads, seqlen, rows, bins, **kw):
    rs = ReadSet(*reads, seqlen, device=0)
    plan = Plan(rs, rows, bins, **kw)
    out = plan.empty_output()
    valid = torch.empty(max(rows.n_rows, 1), dtype=torch.uint8, device=DEV)
    plan.execute(out, valid)
    plan.status()
    return plan, out, valid[:rows.n_rows].cpu().numpy().astype(bool)


def compare(out, valid, exp, ev, rtol=1e-12, atol=0.0):
    np.testing.assert_array_equal(valid, ev.astype(bool))
    mat = out[:, :len(valid)].cpu().numpy().T
    assert mat.shape == exp.shape
    np.testing.assert_allclose(mat, exp, rtol=rtol, atol=atol)


def test_c2_full_size(gpu):
    d = synthetic.c2(device=DEV)
    reg = d["regions"]
    rows = single_rows(reg)
    plan, out, valid = run(d["reads"], d["seqlen"], rows, Bins([("whole", d["n_bins"])]))
    assert rows.n_rows == 10_000 and plan.n_cols == 200
    ix = host_index(d["reads"], d["seqlen"])
    mask = o.Mask.from_ranges(reg["chrom"], reg["start"], reg["end"], reg["strand"])
    exp, ev = o.profile_part(ix, mask, d["n_bins"], nthreads=threads())
    compare(out, valid, exp, ev)
    assert valid.mean() > 0.99


def test_c4_reduced_heavy_rows(gpu):
    d = synthetic.c4(device=DEV, n_regions=20_000, n_reads=20_000_000)
    reg = d["regions"]
    rows = single_rows(reg)
    plan, out, valid = run(d["reads"], d["seqlen"], rows, Bins([("whole", d["n_bins"])]), kernel="lean")
    assert plan.info["pileup_kernel"] == 1  # the lean kernel, as in the bench
    assert plan.heavy_rows() > 0            # Pareto hot peaks go through the heavy slices
    ix = host_index(d["reads"], d["seqlen"])
    mask = o.Mask.from_ranges(reg["chrom"], reg["start"], reg["end"], reg["strand"])
    exp, ev = o.profile_part(ix, mask, d["n_bins"], nthreads=threads())
    compare(out, valid, exp, ev)
    # the general kernel without the heavy path gives the same bits
    plan2, out2, valid2 = run(d["reads"], d["seqlen"], rows, Bins([("whole", d["n_bins"])]), kernel="general",
                              heavy_threshold=0)
    assert plan2.heavy_rows() == 0
    assert torch.equal(out.view(torch.int64), out2.view(torch.int64))
    np.testing.assert_array_equal(valid, valid2)


def closed_form_row_sums(reads, reg):
    """Sum of depth over each region [s, e], exact int64 on the GPU."""
    c, s, e, _ = reads
    c64 = c.to(torch.int64) << 32
    ks, _ = torch.sort(c64 | s.to(torch.int64))
    ke, _ = torch.sort(c64 | e.to(torch.int64))
    ps = torch.zeros(ks.numel() + 1, dtype=torch.int64, device=ks.device)
    pe = torch.zeros_like(ps)
    ps[1:] = torch.cumsum(ks & 0xFFFFFFFF, 0)
    pe[1:] = torch.cumsum(ke & 0xFFFFFFFF, 0)
    del c64
    rc = torch.as_tensor(reg["chrom"], device=ks.device, dtype=torch.int64) << 32

    def C(x):  # sum of depth over positions <= x of the region's chromosome
        base_s = torch.searchsorted(ks, rc)
        hi_s = torch.searchsorted(ks, rc | x, right=True)
        base_e = torch.searchsorted(ke, rc)
        lo_e = torch.searchsorted(ke, rc | x)  # ends < x
        cnt_s, sum_s = hi_s - base_s, ps[hi_s] - ps[base_s]
        cnt_e, sum_e = lo_e - base_e, pe[lo_e] - pe[base_e]
        return cnt_s * (x + 1) - sum_s - (cnt_e * x - sum_e)

    s_ = torch.as_tensor(reg["start"], device=ks.device, dtype=torch.int64)
    e_ = torch.as_tensor(reg["end"], device=ks.device, dtype=torch.int64)
    return C(e_) - C(s_ - 1)


def test_c4_full_size_properties(gpu):
    d = synthetic.c4(device=DEV)
    reg = d["regions"]
    rows = single_rows(reg)
    plan, out, valid = run(d["reads"], d["seqlen"], rows, Bins([("whole", d["n_bins"])]))
    assert out.shape == (1000, 200_000) and plan.info["pileup_kernel"] == 1
    assert plan.heavy_rows() > 0
    two = out * 2.0  # 2-bp bins: 2 x mean is the bin's integer depth sum
    assert bool(torch.all(two == torch.round(two)))
    got = two.sum(0).to(torch.int64)  # exact: < 2^53
    want = closed_form_row_sums(d["reads"], reg)
    ovl = torch.as_tensor(synthetic.n_overlaps(d["reads"], reg, d["width"]), device=DEV)
    np.testing.assert_array_equal(valid, (ovl > 0).cpu().numpy())
    assert bool(torch.all(got == want)), int((got != want).sum())
    assert bool(torch.all(out[:, torch.as_tensor(~valid, device=DEV)] == 0))
    assert valid.mean() > 0.99


def test_c5_reduced_per_base(gpu):
    d = synthetic.c5(device=DEV, n_regions=2_500, n_reads=50_000_000)
    reg = d["regions"]
    rows = single_rows(reg)
    plan, out, valid = run(d["reads"], d["seqlen"], rows, Bins([("whole", 0, 4000)]), out_ld="padded")
    assert plan.info["pileup_kernel"] == 1 and plan.n_cols == 4000 and out.shape == (4000, 2512)
    ix = host_index(d["reads"], d["seqlen"])
    mask = o.Mask.from_ranges(reg["chrom"], reg["start"], reg["end"], reg["strand"])
    exp, ev = o.profile_part(ix, mask, 0, ncol=4000, nthreads=threads())
    compare(out, valid, exp, ev, rtol=0)  # per-base depth: exact


@pytest.mark.parametrize("stat", ["mean", "median"])
def test_c3_reduced(gpu, stat):
    d = synthetic.c3(device=DEV, n_genes=2_500, n_pairs=5_000_000)
    rows = synthetic.rna_rows(d)
    bins = Bins([("upstream", d["flank_bins"]), ("center", d["region_bins"]), ("downstream", d["flank_bins"])],
                flank=d["flank"], stat=stat)
    plan, out, valid = run(d["reads"], d["seqlen"], rows, bins, out_ld=2_600)
    assert plan.n_cols == 600 and plan.info["n_interp_rows"] > 0 and out.shape == (600, 2_600)
    ix = host_index(d["reads"], d["seqlen"])
    exp, ev = o.profile_rows(ix, rows, bins, nthreads=threads())
    compare(out, valid, exp, ev, rtol=1e-9, atol=1e-12)
    assert valid.mean() > 0.5
