"""The row-wave pileup kernel (rcp_kernels.hip rcp_pileup_rows_kernel, plan info
"pileup_kernel" == 3): every wave owns whole rows and walks their parts in windows.  Plans with
multi-range rows (coverageRnaRef's c(flank, exon list, flank), R/coverage.R:79-124) take it under
kernel="auto"; kernel="rows" forces it for any mean plan.  Each case is checked against the CPU
oracle (integer numerators exact, means within 1e-12 relative; R-RNG layouts 1e-9) and bit for
bit against the general kernel on the same plan (kernel="general")."""

import numpy as np
import pytest

from tests.test_gpu_random import CHROM_LEN, check, make_reads, single_rows

pytestmark = pytest.mark.gpu


def _both(reads, seqlen, rows, bins, strand_filter=None, kernel="rows", heavy_threshold=-1, binsum=False):
    from recoup_amd.engine import Plan, ReadSet
    from tests import oracle_rows
    rs = ReadSet(*reads, seqlen, device=0, strand_filter=strand_filter)
    pr = Plan(rs, rows, bins, kernel=kernel, heavy_threshold=heavy_threshold)
    pg = Plan(rs, rows, bins, kernel="general", heavy_threshold=heavy_threshold)
    assert pr.info["pileup_kernel"] == 3 and pg.info["pileup_kernel"] == 0
    a, b = pr.run(binsum=binsum), pg.run(binsum=binsum)
    ix = oracle_rows.index_for(reads, seqlen, strand_filter)
    exp = oracle_rows.profile(oracle_rows.row_coverage(ix, rows), bins)
    np.testing.assert_array_equal(a[1], b[1])
    assert np.array_equal(np.ascontiguousarray(a[0]).view(np.uint64), np.ascontiguousarray(b[0]).view(np.uint64))
    if binsum:
        np.testing.assert_array_equal(a[2], b[2])
    return a, exp, pr


def rna_rows(rng, n_genes, flank=2000, max_exons=9, overlap=True, ignore_strand=True, long_exons=False):
    from recoup_amd.engine import RowTable
    seg_off, ch, st, en, sd, gr = [0], [], [], [], [], []
    for _ in range(n_genes):
        c = int(rng.integers(0, 3))
        pos = int(rng.integers(5000, CHROM_LEN[c] - 80000))
        strand = int(rng.integers(0, 2))
        ex_s, ex_e, p = [], [], pos
        for _ in range(int(rng.integers(1, max_exons + 1))):
            w = int(rng.integers(30, 4000 if long_exons else 600))
            ex_s.append(p)
            ex_e.append(p + w - 1)
            p += w + int(rng.integers(-100 if overlap else 1, 3000))
        gs, ge = min(ex_s), max(ex_e)
        ls, le = (gs - flank, gs - 1) if strand == 0 else (ge + 1, ge + flank)
        rs_, re_ = (ge + 1, ge + flank) if strand == 0 else (gs - flank, gs - 1)
        for s_, e_, g in [(ls, le, 0)] + [(a, b, 1) for a, b in zip(ex_s, ex_e)] + [(rs_, re_, 2)]:
            ch.append(c); st.append(s_); en.append(e_); sd.append(strand); gr.append(g)
        seg_off.append(len(st))
    return RowTable(np.array(seg_off), np.array(ch), np.array(st), np.array(en), np.array(sd),
                    seg_group=np.array(gr), group_is_list=np.array([0, 1, 0, 0]), ignore_strand=ignore_strand)


@pytest.mark.parametrize("stranded", [False, True])
def test_rna_rows_auto(gpu, stranded):
    """coverageRnaRef rows take the row-wave kernel under "auto": flank bins, R-RNG centre
    layouts, exon-list weights (overlapping exons), interpolated short genes (interp kernel)."""
    from recoup_amd.engine import Bins
    rng = np.random.default_rng(41 + stranded)
    reads = make_reads(rng, 150_000, widths=(50, 600))
    rows = rna_rows(rng, 160, ignore_strand=not stranded)
    bins = Bins([("upstream", 50), ("center", 100), ("downstream", 50)], flank=(2000, 2000))
    res, exp, _ = _both(reads, CHROM_LEN, rows, bins, kernel="auto")
    check(res, exp, rtol=1e-9, atol=1e-12)


def test_rna_long_centres_windows(gpu):
    """Exon lists longer than one window (2047 positions): the centre is walked in several
    windows; pieces cut by a window edge are narrowed by the bucket directory."""
    from recoup_amd.engine import Bins
    rng = np.random.default_rng(43)
    reads = make_reads(rng, 200_000, widths=(50, 600))
    rows = rna_rows(rng, 80, long_exons=True, overlap=False)
    for centre in (100, 37, 1000):
        bins = Bins([("upstream", 20), ("center", centre), ("downstream", 20)], flank=(2000, 2000))
        res, exp, _ = _both(reads, CHROM_LEN, rows, bins, kernel="auto")
        check(res, exp, rtol=1e-9, atol=1e-12)


@pytest.mark.parametrize("width,n_bins", [(2000, 150), (2000, 1000), (4000, 200), (1500, 256), (20_000, 333),
                                          (3000, 7)])
def test_single_range_rows_forced(gpu, width, n_bins):
    """Plain ranges through the row-wave kernel: uniform, power-of-two, R-RNG layouts, rows
    longer than a window, bins wider than a lane chunk; NULL rows (negative index, past the
    chromosome end)."""
    from recoup_amd.engine import Bins
    rng = np.random.default_rng(600 + n_bins)
    reads = make_reads(rng, 100_000, star_frac=0.1)
    rows = single_rows(rng, 200, width, edge=True)
    res, exp, _ = _both(reads, CHROM_LEN, rows, Bins([("whole", n_bins)]))
    check(res, exp, rtol=1e-9, atol=1e-12)


def test_per_base_flanks_and_scale(gpu):
    """Per-base flanks + binned centre (profile.R:58-77), the linear scale, and binsum."""
    from recoup_amd.engine import Bins
    rng = np.random.default_rng(47)
    reads = make_reads(rng, 100_000)
    rows = rna_rows(rng, 60, flank=500)
    bins = Bins([("upstream", 0, 500), ("center", 80), ("downstream", 0, 500)], flank=(500, 500), scale=0.37)
    res, exp, _ = _both(reads, CHROM_LEN, rows, bins, binsum=True)
    check(res, exp, rtol=1e-9, atol=1e-12)


@pytest.mark.parametrize("strand_filter", ["+", "-"])
def test_stranded_reads(gpu, strand_filter):
    from recoup_amd.engine import Bins
    rng = np.random.default_rng(53)
    reads = make_reads(rng, 80_000)
    rows = single_rows(rng, 120, 2000)
    res, exp, _ = _both(reads, CHROM_LEN, rows, Bins([("whole", 200)]), strand_filter=strand_filter)
    check(res, exp)


def test_heavy_rows(gpu):
    """Skewed rows piled by the heavy slice kernel first, single-range and exon lists."""
    from recoup_amd.engine import Bins
    rng = np.random.default_rng(59)
    reads = make_reads(rng, 200_000, widths=(100, 200))
    rows = single_rows(rng, 100, 2000)
    res, exp, plan = _both(reads, CHROM_LEN, rows, Bins([("whole", 100)]), heavy_threshold=16)
    check(res, exp)
    assert plan.heavy_rows() > 0
    rows = rna_rows(rng, 60)
    bins = Bins([("upstream", 50), ("center", 100), ("downstream", 50)], flank=(2000, 2000))
    res, exp, _ = _both(reads, CHROM_LEN, rows, bins, heavy_threshold=16)
    check(res, exp, rtol=1e-9, atol=1e-12)


def test_repeated_executions_and_kernel_choice(gpu):
    """The row counters are reset by the last workgroup: one plan executed repeatedly gives the
    same bits; medians and single-range plans keep their kernels under "auto"."""
    from recoup_amd.engine import Bins, Plan, ReadSet
    rng = np.random.default_rng(61)
    reads = make_reads(rng, 60_000)
    rs = ReadSet(*reads, CHROM_LEN, device=0)
    rows = rna_rows(rng, 300)
    bins = Bins([("upstream", 50), ("center", 100), ("downstream", 50)], flank=(2000, 2000))
    plan = Plan(rs, rows, bins)
    assert plan.info["pileup_kernel"] == 3
    first = plan.run()
    for _ in range(3):
        again = plan.run()
        assert np.array_equal(np.ascontiguousarray(again[0]).view(np.uint64),
                              np.ascontiguousarray(first[0]).view(np.uint64))
    med = Bins([("upstream", 50), ("center", 100), ("downstream", 50)], flank=(2000, 2000), stat="median")
    assert Plan(rs, rows, med).info["pileup_kernel"] == 0
    single = single_rows(rng, 50, 2000)
    assert Plan(rs, single, Bins([("whole", 150)])).info["pileup_kernel"] == 0
    assert Plan(rs, single, Bins([("whole", 1000)]), kernel="lean").info["pileup_kernel"] == 1
    assert Plan(rs, rows, bins, kernel="general").info["pileup_kernel"] == 0


def test_row_major_staging(gpu):
    """Tiles staged as bin numerators in the HBM row-major stage -- C3's 600 columns and a wide
    plan (4100 columns of per-base flanks): the same bits as the general kernel, NULL rows and
    interpolated short genes included."""
    from recoup_amd.engine import Bins
    rng = np.random.default_rng(67)
    reads = make_reads(rng, 150_000, widths=(50, 600))
    rows = rna_rows(rng, 203)
    c3 = Bins([("upstream", 50), ("center", 500), ("downstream", 50)], flank=(2000, 2000), scale=0.61)
    res, exp, plan = _both(reads, CHROM_LEN, rows, c3, kernel="auto")
    check(res, exp, rtol=1e-9, atol=1e-12)
    wide = Bins([("upstream", 0, 2000), ("center", 100), ("downstream", 0, 2000)], flank=(2000, 2000))
    res, exp, plan = _both(reads, CHROM_LEN, rows, wide, kernel="auto")
    assert plan.info["lds_bytes"] <= 160 * 1024  # (row-major staging in HBM: the waves' windows only)
    check(res, exp, rtol=1e-9, atol=1e-12)


@pytest.mark.parametrize("stranded", [False, True])
def test_folded_locate(gpu, stranded):
    """Row-wave plans search their rows' read ranges in the pileup kernel (plan dev.fold: no
    locate launch) unless the caller asks for the heavy path: NA seqlengths (the group's hits'
    last end decides, R/coverage.R:217-222), NULL rows, interpolated genes both from the HBM stage
    and -- with binsum -- piled again by the interpolation kernel from the ranges the pileup wrote,
    and one plan executed with and without binsum in turn; the same bits as the located plan
    (heavy_threshold 16) and the general kernel."""
    from recoup_amd.engine import Bins, Plan, ReadSet
    rng = np.random.default_rng(71 + stranded)
    reads = make_reads(rng, 120_000, widths=(50, 600), star_frac=0.1)
    rows = rna_rows(rng, 150, ignore_strand=not stranded)
    bins = Bins([("upstream", 50), ("center", 300), ("downstream", 50)], flank=(2000, 2000))
    for seqlen in (CHROM_LEN, np.array([-1, CHROM_LEN[1], -1], np.int64)):
        res, exp, plan = _both(reads, seqlen, rows, bins, kernel="auto")
        check(res, exp, rtol=1e-9, atol=1e-12)
        assert plan.heavy_rows() == 0
        located = Plan(ReadSet(*reads, seqlen, device=0), rows, bins, heavy_threshold=16)
        ref = located.run(binsum=True)
        for binsum in (True, False, True):
            got = plan.run(binsum=binsum)
            np.testing.assert_array_equal(got[1], ref[1])
            assert np.array_equal(np.ascontiguousarray(got[0]).view(np.uint64),
                                  np.ascontiguousarray(ref[0]).view(np.uint64))
            if binsum:
                np.testing.assert_array_equal(got[2], ref[2])
