"""Every BASELINE.json configuration under -m gpu (the bench's workloads, synthetic.py):

  C2  full size: 10k TSS +-2 kb, 200 bins, 10M reads                  vs the CPU oracle
  C4  reduced:   20k peaks, 20M reads, Pareto hot peaks (heavy path)    vs the CPU oracle
  C4  full size: 200k peaks x 1000 bins, 200M reads                     size-independent properties
  C5  reduced:   2.5k regions x 4000 bp per base, 50M reads             vs the CPU oracle
  C5  full size: 25k regions x 4000 bp per base, 500M reads             closed-form row sums + oracle rows
  C3  reduced:   2.5k genes (exon lists + flanks), 5M read pairs         vs the CPU oracle
  C3  full size: 25k genes, 50M read pairs                              oracle on a row sample

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


def reads_overlapping(reads, chrom, lo, hi):
    """The reads overlapping any span [lo, hi] of a chromosome (device mask): spans sorted by
    (chrom, lo), each read's last span starting at or before its end, and the prefix max of
    the span ends up to it (same chromosome) -- the reads an oracle needs for those rows."""
    c, s, e, _ = reads
    dev = c.device
    key_lo = (torch.as_tensor(chrom, device=dev, dtype=torch.int64) << 32) | torch.as_tensor(lo, device=dev,
                                                                                           dtype=torch.int64)
    key_hi = (torch.as_tensor(chrom, device=dev, dtype=torch.int64) << 32) | torch.as_tensor(hi, device=dev,
                                                                                           dtype=torch.int64)
    order = torch.argsort(key_lo)
    key_lo, key_hi = key_lo[order], key_hi[order]
    cm = torch.cummax(key_hi, 0).values
    c64 = c.to(torch.int64) << 32
    idx = torch.searchsorted(key_lo, c64 | e.to(torch.int64), right=True) - 1
    ok = idx >= 0
    best = cm[idx.clamp(min=0)]
    return ok & ((best >> 32) == c.to(torch.int64)) & ((best & 0xFFFFFFFF) >= s.to(torch.int64))


def sample_index(reads, seqlen, mask):
    """The oracle's read index of the reads `mask` selects, in (chrom, start) order."""
    c, s, e, st = (x[mask] for x in reads)
    order = torch.argsort((c.to(torch.int64) << 32) | s.to(torch.int64))
    return o.Index(*[x[order].cpu().numpy() for x in (c, s, e, st)], seqlen)


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


def test_c5_full_size(gpu):
    """BASELINE config 5 at its stated size (25k x 4000 bp per base, 500M reads): every row's
    per-base depth sums to the closed-form overlap sum exactly, a row is
    valid iff a read overlaps it, and the first 2,500 rows equal the oracle's per-base depth bit
    for bit (R/profile.R:100-151, R/coverage.R:176-226)."""
    d = synthetic.c5(device=DEV)
    reg = d["regions"]
    rows = single_rows(reg)
    plan, out, valid = run(d["reads"], d["seqlen"], rows, Bins([("whole", 0, 4000)]), out_ld="padded")
    assert plan.info["pileup_kernel"] == 1 and out.shape[0] == 4000 and rows.n_rows == 25_000
    assert d["reads"][0].numel() == 500_000_000
    got = out[:, :rows.n_rows].sum(0).to(torch.int64)  # exact: integer depths, sums < 2^53
    want = closed_form_row_sums(d["reads"], reg)
    assert bool(torch.all(got == want)), int((got != want).sum())
    ovl = synthetic.n_overlaps(d["reads"], reg, d["width"])
    np.testing.assert_array_equal(valid, ovl > 0)
    m = 2_500
    sel = reads_overlapping(d["reads"], reg["chrom"][:m], reg["start"][:m], reg["end"][:m])
    ix = sample_index(d["reads"], d["seqlen"], sel)
    mask = o.Mask.from_ranges(reg["chrom"][:m], reg["start"][:m], reg["end"][:m], reg["strand"][:m])
    exp, ev = o.profile_part(ix, mask, 0, ncol=4000, nthreads=threads())
    mat = out[:, :m].cpu().numpy().T
    np.testing.assert_array_equal(valid[:m], ev.astype(bool))
    assert np.array_equal(mat.view(np.int64), np.ascontiguousarray(exp).view(np.int64))


def test_c3_full_size(gpu):
    """BASELINE config 3 at its stated size (25k genes: flank | exon list | flank rows, 50M read
    pairs = 100M mate alignments, spliced mates split into blocks): the oracle's coverageRnaRef
    profile (R/coverage.R:79-124 merged, R/profile.R:13-81) on a sample of 2,000 genes spread over
    the table -- integer-layout bins within 1e-12, R-RNG / interpolated rows within 1e-9."""
    d = synthetic.c3(device=DEV)
    rows = synthetic.rna_rows(d)
    bins = Bins([("upstream", d["flank_bins"]), ("center", d["region_bins"]), ("downstream", d["flank_bins"])],
                flank=d["flank"])
    plan, out, valid = run(d["reads"], d["seqlen"], rows, bins, out_ld="padded")
    assert rows.n_rows == 25_000 and plan.n_cols == 600 and plan.info["pileup_kernel"] == 3
    pick = np.linspace(0, rows.n_rows - 1, 2_000).astype(np.int64)
    seg = [np.arange(rows.seg_off[r], rows.seg_off[r + 1]) for r in pick]
    sub = RowTable(np.concatenate([[0], np.cumsum([len(x) for x in seg])]), rows.chrom[np.concatenate(seg)],
                   rows.start[np.concatenate(seg)], rows.end[np.concatenate(seg)], rows.strand[np.concatenate(seg)],
                   seg_group=rows.seg_group[np.concatenate(seg)], group_is_list=rows.group_is_list,
                   ignore_strand=rows.ignore_strand)
    span_lo = np.array([rows.start[x].min() for x in seg])
    span_hi = np.array([rows.end[x].max() for x in seg])
    sel = reads_overlapping(d["reads"], rows.chrom[rows.seg_off[pick]], np.maximum(span_lo, 1), span_hi)
    ix = sample_index(d["reads"], d["seqlen"], sel)
    exp, ev = o.profile_rows(ix, sub, bins, nthreads=threads())
    mat = out[:, torch.as_tensor(pick, device=DEV)].cpu().numpy().T
    np.testing.assert_array_equal(valid[pick], ev.astype(bool))
    np.testing.assert_allclose(mat, exp, rtol=1e-9, atol=1e-12)
    assert valid.mean() > 0.5


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
