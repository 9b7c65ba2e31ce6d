"""Randomised GPU-vs-oracle parity over the reference's edge cases.

Each case builds seeded reads and rows, runs the HIP path through the C ABI and compares
with the CPU oracle: row validity (the reference's NULL rows) and integer numerators
bit-exact, means within 1e-12 relative, interpolated / median values within 1e-9
(north_star's bar for means is 1e-6)."""
import os

import numpy as np
import pytest

from tests import oracle_rows

pytestmark = pytest.mark.gpu

CHROM_LEN = np.array([400_000, 250_000, 90_000], dtype=np.int64)


def make_reads(rng, n, widths=(20, 400), chroms=3, star_frac=0.0):
    chrom = rng.integers(0, chroms, n).astype(np.int32)
    start = np.empty(n, dtype=np.int64)
    for c in range(chroms):
        m = chrom == c
        # clustered + uniform starts (hot spots exercise deep pileups)
        k = int(m.sum())
        centers = rng.integers(1000, CHROM_LEN[c] - 1000, 20)
        hot = rng.random(k) < 0.4
        s = rng.integers(1, CHROM_LEN[c] - widths[1], k)
        s[hot] = centers[rng.integers(0, 20, hot.sum())] + rng.integers(-600, 600, hot.sum())
        start[m] = np.clip(s, 1, CHROM_LEN[c] - widths[1])
    width = rng.integers(widths[0], widths[1] + 1, n)
    end = start + width - 1
    strand = rng.integers(0, 2, n).astype(np.int8)
    if star_frac:
        strand[rng.random(n) < star_frac] = 2
    return chrom, start.astype(np.int32), end.astype(np.int32), strand


def single_rows(rng, R, width, chroms=3, strands=(0, 1, 2), edge=False):
    from recoup_amd.engine import RowTable
    chrom = rng.integers(0, chroms, R).astype(np.int32)
    s = np.array([rng.integers(1, CHROM_LEN[c] - width) for c in chrom], dtype=np.int64)
    if edge:
        s[:3] = [-50, 0, 1]                       # negative index -> NULL; 0 -> dropped index
        s[3] = CHROM_LEN[chrom[3]] - width // 2     # runs past the chromosome -> NULL
    e = s + width - 1
    st = rng.choice(np.array(strands, dtype=np.int8), R)
    return RowTable.from_ranges(chrom, s, e, st)


def run_case(reads, seqlen, rows, bins, strand_filter=None, binsum=False, **plan_kw):
    from recoup_amd.engine import Plan, ReadSet
    rs = ReadSet(*reads, seqlen, device=0, strand_filter=strand_filter)
    plan = Plan(rs, rows, bins, **plan_kw)
    res = plan.run(binsum=binsum)
    ix = oracle_rows.index_for(reads, seqlen, strand_filter)
    cov = oracle_rows.row_coverage(ix, rows)
    exp, ev = oracle_rows.profile(cov, bins)
    return res, (exp, ev, cov)


def check(res, expected, rtol=1e-12, atol=0.0):
    mat, valid = res[0], res[1]
    exp, ev = expected[0], expected[1]
    np.testing.assert_array_equal(valid, ev)
    assert mat.shape == exp.shape
    np.testing.assert_allclose(mat, exp, rtol=rtol, atol=atol)


@pytest.mark.parametrize("n_bins", [1, 7, 64, 150, 1000])
def test_single_range_bins(gpu, n_bins):
    from recoup_amd.engine import Bins
    rng = np.random.default_rng(100 + n_bins)
    reads = make_reads(rng, 60_000, star_frac=0.1)
    rows = single_rows(rng, 300, 2000)
    res, exp = run_case(reads, CHROM_LEN, rows, Bins([("whole", n_bins)]), binsum=True)
    check(res, exp)
    # bin numerators are integer sums: exact
    cov = exp[2]
    from oracle import oracle as o
    for r in range(0, 300, 37):
        if cov[r] is None:
            continue
        ref = o.split_vector(cov[r].astype(float), n_bins, stat="mean")
        sizes = _layout_sizes(2000, n_bins)
        np.testing.assert_array_equal(res[2][r], np.rint(ref * sizes).astype(np.int64))


def _layout_sizes(L, n):
    from oracle import oracle as o
    bs, dif = divmod(L, n)
    sizes = np.full(n, bs)
    if dif:
        o.set_seed(42)
        sizes[o.sample_int(n, dif) - 1] += 1
    return sizes


def test_per_base_and_edges(gpu):
    from recoup_amd.engine import Bins
    rng = np.random.default_rng(7)
    reads = make_reads(rng, 80_000)
    rows = single_rows(rng, 200, 3000, edge=True)
    # row 1 starts at 0 -> one position shorter: not valid as a per-base row of 3000; use bins
    res, exp = run_case(reads, CHROM_LEN, rows, Bins([("whole", 100)]))
    check(res, exp)
    assert not res[1][0] and not res[1][3]  # negative index, past the chromosome


def test_na_seqlengths(gpu):
    from recoup_amd.engine import Bins
    rng = np.random.default_rng(11)
    reads = make_reads(rng, 40_000)
    rows = single_rows(rng, 300, 1500)
    seqlen = np.array([-1, -1, -1], dtype=np.int64)  # Rle spans only to the hits' max end
    res, exp = run_case(reads, seqlen, rows, Bins([("whole", 30)]))
    check(res, exp)


@pytest.mark.parametrize("strand_filter", [None, "+", "-"])
def test_stranded(gpu, strand_filter):
    from recoup_amd.engine import Bins, RowTable
    rng = np.random.default_rng(21)
    reads = make_reads(rng, 50_000, star_frac=0.2)
    r0 = single_rows(rng, 250, 1200)
    rows = RowTable(r0.seg_off, r0.chrom, r0.start, r0.end, r0.strand, ignore_strand=False)
    res, exp = run_case(reads, CHROM_LEN, rows, Bins([("whole", 40)]), strand_filter=strand_filter)
    check(res, exp)


def test_rna_multi_exon(gpu):
    """coverageRnaRef rows: flank | exon list (reads counted once per exon hit) | flank."""
    from recoup_amd.engine import Bins, RowTable
    rng = np.random.default_rng(5)
    reads = make_reads(rng, 120_000, widths=(50, 600))
    seg_off, ch, st, en, sd, gr = [0], [], [], [], [], []
    for g in range(120):
        c = int(rng.integers(0, 3))
        pos = int(rng.integers(5000, CHROM_LEN[c] - 60000))
        strand = int(rng.integers(0, 2))
        ne = int(rng.integers(1, 9))
        ex_s, ex_e, p = [], [], pos
        for _ in range(ne):
            w = int(rng.integers(30, 600))
            ex_s.append(p)
            ex_e.append(p + w - 1)
            p += w + int(rng.integers(-100, 3000))  # some overlapping exons
        gs, ge = min(ex_s), max(ex_e)
        f1, f2 = 2000, 2000
        ls, le = (gs - f1, gs - 1) if strand == 0 else (ge + 1, ge + f1)
        rs_, re_ = (ge + 1, ge + f2) if strand == 0 else (gs - f2, gs - 1)
        for s, e, grp in [(ls, le, 0)] + [(a, b, 1) for a, b in zip(ex_s, ex_e)] + [(rs_, re_, 2)]:
            ch.append(c); st.append(s); en.append(e); sd.append(strand); gr.append(grp)
        seg_off.append(len(st))
    rows = RowTable(np.array(seg_off), np.array(ch), np.array(st), np.array(en), np.array(sd),
                    seg_group=np.array(gr), group_is_list=np.array([0, 1, 0, 0]))
    for stat in ("mean", "median"):
        bins = Bins([("upstream", 50), ("center", 100), ("downstream", 50)], flank=(2000, 2000), stat=stat)
        res, exp = run_case(reads, CHROM_LEN, rows, bins)
        check(res, exp, rtol=1e-9, atol=1e-12)


def test_genebody_unequal_interp(gpu):
    """Unequal rows: binned flanks, center bins with RNG layouts, spline / neighborhood rows."""
    from recoup_amd.engine import Bins, RowTable
    rng = np.random.default_rng(9)
    reads = make_reads(rng, 100_000)
    R = 220
    chrom = rng.integers(0, 3, R).astype(np.int32)
    width = np.concatenate([rng.integers(20, 140, 40), rng.integers(140, 40_000, R - 40)])
    s = np.array([rng.integers(3000, CHROM_LEN[c] - 45000) for c in chrom])
    strand = rng.integers(0, 2, R).astype(np.int8)
    f1, f2 = 1000, 1500
    gs = np.where(strand == 0, s - f1, s - f2)
    ge = np.where(strand == 0, s + width - 1 + f2, s + width - 1 + f1)
    rows = RowTable.from_ranges(chrom, gs, ge, strand)
    for interp in ("auto", "spline", "neighborhood", "linear"):
        bins = Bins([("upstream", 20), ("center", 150), ("downstream", 30)], flank=(f1, f2), interp=interp)
        if interp == "neighborhood":
            # R errors for tiny slices; keep the rows where R's neighborhood is defined
            keep = width >= 60
            rows_k = RowTable.from_ranges(chrom[keep], gs[keep], ge[keep], strand[keep])
            res, exp = run_case(reads, CHROM_LEN, rows_k, bins)
        else:
            res, exp = run_case(reads, CHROM_LEN, rows, bins)
        check(res, exp, rtol=1e-9, atol=1e-12)
    # per-base flanks (flankBinSize = 0) with a binned center
    bins = Bins([("upstream", 0, f1), ("center", 100), ("downstream", 0, f2)], flank=(f1, f2))
    res, exp = run_case(reads, CHROM_LEN, rows, bins)
    check(res, exp, rtol=1e-9, atol=1e-12)


@pytest.mark.parametrize("n_bins", [201, 150, 1000])
def test_spline_rows_bit_exact(gpu, n_bins):
    """Interpolated rows (length < bins) equal R's spline() bit for bit: widths whose output
    points fall exactly on knots (n = 201, L = 101 / 51 / 41 / 21 / 11 / 5: points 1/2, 1/4,
    ... apart), where spline_eval keeps the previous interval and evaluates at dx = 1, plus
    widths 2 and 3 (the n < 4 branches) and a spread of others."""
    from recoup_amd.engine import Bins
    rng = np.random.default_rng(31 + n_bins)
    reads = make_reads(rng, 60_000, widths=(20, 200))
    widths = [2, 3, 4, 5, 11, 21, 41, 51, 101, 149, 150, 200]
    widths = [w for w in widths if w < n_bins] + list(rng.integers(2, min(n_bins, 700), 12))
    from recoup_amd.engine import RowTable
    R = len(widths) * 6
    chrom = rng.integers(0, 3, R).astype(np.int32)
    w = np.repeat(np.array(widths, dtype=np.int64), 6)
    # starts inside the hot spots' span so most rows carry signal
    s = np.array([rng.integers(2000, CHROM_LEN[c] - 2000) for c in chrom], dtype=np.int64)
    rows = RowTable.from_ranges(chrom, s, s + w - 1, rng.integers(0, 2, R).astype(np.int8))
    res, exp = run_case(reads, CHROM_LEN, rows, Bins([("whole", n_bins)], interp="spline"))
    np.testing.assert_array_equal(res[1], exp[1])
    np.testing.assert_array_equal(res[0], exp[0])


def test_chunk_edges_all_inside(gpu):
    """A centre part of 8 column chunks whose every edge lies inside the row (flanks on both
    sides): 2 + 16 locate searches per row, more than one lockstep round per lane."""
    from recoup_amd.engine import Bins
    rng = np.random.default_rng(17)
    reads = make_reads(rng, 120_000, widths=(50, 300))
    rows = single_rows(rng, 120, 9000)
    for n_bins in (4000, 2900):  # 2 bp bins (lean kernel), R-RNG layout (general kernel)
        res, exp = run_case(reads, CHROM_LEN, rows, Bins([("center", n_bins)], flank=(500, 500)))
        check(res, exp)


def test_long_rows_chunked(gpu):
    """Rows longer than one chunk: per-base (chunked columns) and coarse bins."""
    from recoup_amd.engine import Bins
    rng = np.random.default_rng(13)
    reads = make_reads(rng, 150_000)
    rows = single_rows(rng, 40, 20_000)
    res, exp = run_case(reads, CHROM_LEN, rows, Bins([("whole", 0, 20_000)]))
    check(res, exp)
    res, exp = run_case(reads, CHROM_LEN, rows, Bins([("whole", 333)]))
    check(res, exp)


def test_heavy_rows_match(gpu):
    """Skewed rows through the heavy split path give the same matrix as the oracle."""
    from recoup_amd.engine import Bins
    rng = np.random.default_rng(17)
    reads = make_reads(rng, 200_000, widths=(100, 200))
    rows = single_rows(rng, 100, 2000)
    res, exp = run_case(reads, CHROM_LEN, rows, Bins([("whole", 100)]), heavy_threshold=16)
    res_m, exp_m = run_case(reads, CHROM_LEN, rows, Bins([("whole", 100)], stat="median"), heavy_threshold=16)
    check(res, exp)
    check(res_m, exp_m, rtol=1e-9, atol=1e-12)


def test_heavy_duplicate_stacks_match(gpu):
    """Hot rows made of PCR-duplicate stacks (thousands of reads on one start, equal widths):
    the heavy path merges a wave's equal positions into one LDS add per run, both strands,
    per-base and binned, plus stranded (ignore.strand = FALSE) multi-stream rows."""
    from recoup_amd.engine import Bins, RowTable
    rng = np.random.default_rng(29)
    n = 120_000
    chrom = np.zeros(n, np.int32)
    stacks = rng.integers(5000, 5400, 40)                        # 40 duplicate stacks near one spot
    start = np.where(rng.random(n) < 0.8, stacks[rng.integers(0, 40, n)], rng.integers(1, 900_000, n))
    width = np.where(rng.random(n) < 0.9, 150, rng.integers(30, 300, n))
    reads = (chrom, start.astype(np.int64), (start + width - 1).astype(np.int64),
             rng.integers(0, 3, n).astype(np.int8))
    seqlen = np.array([1_000_000], np.int64)
    s0 = np.array([4000, 4100, 4500, 5100, 3000, 5300, 100_000], np.int64)
    rows = RowTable.from_ranges(np.zeros(7, np.int32), s0, s0 + 1999, np.array([0, 1, 2, 1, 0, 1, 2], np.int8))
    for bins in (Bins([("whole", 100)]), Bins([("whole", 0, 2000)])):
        res, exp = run_case(reads, seqlen, rows, bins, heavy_threshold=16)
        check(res, exp)
    stranded = RowTable.from_ranges(np.zeros(7, np.int32), s0, s0 + 1999,
                                    np.array([0, 1, 2, 1, 0, 1, 2], np.int8), ignore_strand=False)
    res, exp = run_case(reads, seqlen, stranded, Bins([("whole", 250)]), heavy_threshold=16)
    check(res, exp)


def test_heavy_repeated_executions(gpu):
    """Each execution's locate kernel clears the heavy slots the previous call left and zeroes
    the previous call's status words (executions alternate between two sets; there is no reset
    launch and no clear after the pileup): one plan run repeatedly, with validity-only and
    coverage calls in between, gives the oracle's matrix every time."""
    from recoup_amd.engine import Bins, Plan, ReadSet
    rng = np.random.default_rng(31)
    reads = make_reads(rng, 200_000, widths=(100, 200))
    rows = single_rows(rng, 100, 2000)
    rs = ReadSet(*reads, CHROM_LEN, device=0)
    plan = Plan(rs, rows, Bins([("whole", 100)]), heavy_threshold=16)
    ix = oracle_rows.index_for(reads, CHROM_LEN)
    cov = oracle_rows.row_coverage(ix, rows)
    exp = oracle_rows.profile(cov, Bins([("whole", 100)]))
    for k in range(3):
        check(plan.run(), exp)
        if k == 0:
            np.testing.assert_array_equal(plan.validity(), exp[1])
        if k == 1:
            got = plan.coverage()
            for g, e in zip(got, cov):
                assert (g is None) == (e is None)
                if e is not None:
                    np.testing.assert_array_equal(g, e)


def test_calc_coverage_csr(gpu):
    from recoup_amd.engine import Plan, ReadSet
    rng = np.random.default_rng(3)
    reads = make_reads(rng, 70_000)
    rows = single_rows(rng, 150, 5000, edge=True)
    rs = ReadSet(*reads, CHROM_LEN, device=0)
    got = Plan(rs, rows, None).coverage()
    ix = oracle_rows.index_for(reads, CHROM_LEN)
    exp = oracle_rows.row_coverage(ix, rows)
    for g, e in zip(got, exp):
        if e is None:
            assert g is None
        else:
            np.testing.assert_array_equal(g, e)


def test_rounding_sample_kind(gpu):
    """RNGkind(sample.kind = "Rounding") (pre-3.6 R) bin layouts."""
    from recoup_amd.engine import Bins
    from oracle import oracle as o
    rng = np.random.default_rng(23)
    reads = make_reads(rng, 30_000)
    rows = single_rows(rng, 100, 2000)
    from recoup_amd.engine import Plan, ReadSet
    rs = ReadSet(*reads, CHROM_LEN, device=0)
    mat, valid = Plan(rs, rows, Bins([("whole", 150)], rng_kind="Rounding")).run()
    ix = oracle_rows.index_for(reads, CHROM_LEN)
    cov = oracle_rows.row_coverage(ix, rows)
    exp = o._bin_matrix(cov, 150, "mean", "auto", None, None, 1.0, "Rounding")
    np.testing.assert_allclose(mat, exp, rtol=1e-12, atol=0)


def test_empty_inputs(gpu):
    from recoup_amd.engine import Bins, Plan, ReadSet, RowTable
    rs = ReadSet(np.zeros(0, np.int32), np.zeros(0, np.int32), np.zeros(0, np.int32), np.zeros(0, np.int8),
                 CHROM_LEN, device=0)
    rows = single_rows(np.random.default_rng(1), 20, 1000)
    mat, valid = Plan(rs, rows, Bins([("whole", 10)])).run()
    assert not valid.any() and not mat.any()
    empty = RowTable(np.zeros(1, np.int64), np.zeros(0, np.int32), np.zeros(0, np.int32), np.zeros(0, np.int32),
                     np.zeros(0, np.int8))
    mat, valid = Plan(rs, empty, Bins([("whole", 10)])).run()
    assert mat.shape == (0, 10)


@pytest.mark.parametrize("kernel,n_bins,stat", [("auto", 1000, "mean"), ("general", 150, "mean"),
                                                ("general", 64, "median"), ("auto", 0, "mean")])
def test_output_leading_dimension(gpu, kernel, n_bins, stat):
    """rcp_plan_opts.out_ld: a padded column stride (multiple of 16 rows) or any ld >= n_rows
    gives the same bits in columns [:, :n_rows] as the plain R layout; interpolated rows
    (700-bp rows, 1000 bins) write through the same stride.  The padding is never written."""
    import torch
    from recoup_amd.engine import Bins, Plan, ReadSet
    rng = np.random.default_rng(91)
    reads = make_reads(rng, 80_000)
    rows = single_rows(rng, 333, 2000)
    rows.end[::7] = rows.start[::7] + 699  # L < n bins: the interpolation kernel
    rs = ReadSet(*reads, CHROM_LEN, device=0)
    bins = Bins([("whole", n_bins)], stat=stat) if n_bins else Bins([("whole", 0, 2000)])
    if n_bins == 0:
        rows.end[::7] = rows.start[::7] + 1999
    ref = Plan(rs, rows, bins, kernel=kernel).run()
    for ld in ("padded", 341, 400):
        plan = Plan(rs, rows, bins, kernel=kernel, out_ld=ld)
        out = torch.full((plan.n_cols, plan.out_ld), -7.0, dtype=torch.float64, device="cuda:0")
        valid = torch.empty(333, dtype=torch.uint8, device="cuda:0")
        plan.execute(out, valid)
        plan.status()
        assert plan.out_ld == (336 if ld == "padded" else ld)
        got = out[:, :333].cpu().numpy().T
        assert np.array_equal(got.view(np.uint64), ref[0].view(np.uint64))
        np.testing.assert_array_equal(valid.cpu().numpy().astype(bool), ref[1])
        assert bool(torch.all(out[:, 333:] == -7.0))


@pytest.mark.parametrize("ignore_strand", [True, False])
def test_coordinates_near_int32_max(gpu, ignore_strand):
    """A chromosome of 2,147,483,000 bp (just under the int32 coordinate limit the C ABI
    states): reads and rows at its far end, a row ending on its last base (valid), one running
    past it (NULL, coverage.R:217-222), a hot spot taking the heavy path, a second small
    chromosome; lean (2-bp bins), general (40 bins) and per-base plans, merged and stranded
    read layouts, known and NA seqlengths -- all against the oracle."""
    from recoup_amd.engine import Bins, RowTable
    rng = np.random.default_rng(47)
    L0 = 2_147_483_000
    n0, n1, nh = 60_000, 20_000, 20_000
    s0 = rng.integers(L0 - 1_000_000, L0 - 179, n0)
    sh = rng.integers(L0 - 500_000, L0 - 499_000, nh)             # hot spot: heavy rows
    s1 = rng.integers(1, 99_000, n1)
    start = np.concatenate([s0, sh, s1]).astype(np.int64)
    width = rng.integers(20, 181, start.size)
    end = np.minimum(start + width - 1, np.where(np.arange(start.size) < n0 + nh, L0, 100_000))
    chrom = np.concatenate([np.zeros(n0 + nh, np.int32), np.ones(n1, np.int32)])
    strand = rng.integers(0, 3, start.size).astype(np.int8)
    reads = (chrom, start.astype(np.int32), end.astype(np.int32), strand)
    R = 300
    rc = np.zeros(R, np.int32)
    rs_ = rng.integers(L0 - 990_000, L0 - 2000, R).astype(np.int64)
    rs_[:8] = L0 - 500_800 + 100 * np.arange(8)                    # on the hot spot
    rs_[8] = L0 - 1999                                             # ends on the last base
    rs_[9] = L0 - 1500                                             # runs past the chromosome
    rc[10:20] = 1
    rs_[10:20] = rng.integers(1, 97_000, 10)
    st = rng.integers(0, 3, R).astype(np.int8)
    rows = RowTable.from_ranges(rc, rs_, rs_ + 1999, st, ignore_strand=ignore_strand)
    for seqlen in (np.array([L0, 100_000], np.int64), np.array([-1, -1], np.int64)):
        for bins in (Bins([("whole", 1000)]), Bins([("whole", 40)]), Bins([("whole", 0, 2000)])):
            res, exp = run_case(reads, seqlen, rows, bins, heavy_threshold=64)
            check(res, exp)
            if seqlen[0] > 0:
                assert res[1][8] and not res[1][9]


@pytest.mark.parametrize("uniform", [True, False], ids=["one_width", "many_widths"])
def test_fold_plans_and_cooperative_rows(gpu, uniform):
    """Small single-range tables in the merged layout run the general kernel FOLDED: each
    workgroup searches its rows' and chunk's read ranges itself (no locate launch), and a row
    whose chunk holds more than 8192 candidate reads is piled by the whole workgroup (no heavy
    slices).  C4's shape (2-bp bins in two column chunks), per-base and 20-bp bins; rows on both
    strands over a 60k-read pile; NA seqlengths; repeated executions.  Bit-equal to the oracle
    and to the same plan on the locate + heavy-slice path."""
    from recoup_amd.engine import Bins, Plan, ReadSet, RowTable
    rng = np.random.default_rng(77 + uniform)
    base = make_reads(rng, 150_000, widths=(150, 150) if uniform else (40, 400))
    k = 60_000
    hs = (200_000 + rng.integers(0, 1500, k)).astype(np.int32)
    hw = np.full(k, 150) if uniform else rng.integers(40, 400, k)
    reads = (np.r_[base[0], np.zeros(k, np.int32)], np.r_[base[1], hs], np.r_[base[2], (hs + hw - 1).astype(np.int32)],
             np.r_[base[3], rng.integers(0, 3, k).astype(np.int8)])
    r0 = single_rows(rng, 300, 2000, edge=True)
    r0.start[1], r0.end[1] = 1, 2000  # (a start at 0 shortens its row: not a per-base row of 2000)
    hot = (199_000 + rng.integers(-800, 1200, 8)).astype(np.int64)
    rows = RowTable.from_ranges(np.r_[r0.chrom, np.zeros(8, np.int32)], np.r_[r0.start, hot],
                                np.r_[r0.end, hot + 1999], np.r_[r0.strand, np.array([0, 1, 2, 1, 0, 1, 2, 1], np.int8)])
    for seqlen in (CHROM_LEN, np.full(3, -1, np.int64)):
        rs = ReadSet(*reads, seqlen, device=0)
        ix = oracle_rows.index_for(reads, seqlen)
        cov = oracle_rows.row_coverage(ix, rows)
        for bins in (Bins([("whole", 1000)]), Bins([("whole", 0, 2000)]), Bins([("whole", 100)])):
            fold = Plan(rs, rows, bins, kernel="general")
            assert fold.info["fold"] == 1 and fold.info["pileup_kernel"] == 0, fold.info
            slices = Plan(rs, rows, bins, kernel="general", heavy_threshold=4096)
            assert slices.info["fold"] == 0
            exp = oracle_rows.profile(cov, bins)
            ref = slices.run()
            assert slices.heavy_rows() > 0  # (the pile is skewed enough for the slice path)
            for _ in range(3):  # (status words alternate between executions)
                got = fold.run()
                check(got, exp)
                np.testing.assert_array_equal(got[1], ref[1])
                assert np.array_equal(got[0].view(np.uint64), ref[0].view(np.uint64))
            np.testing.assert_array_equal(fold.validity(), exp[1])
