"""The bin-difference pileup kernel (rcp_kernels.hip rcp_pileup_bins_kernel, plan info
"pileup_kernel" == 4).

Mean plans of one binned part whose single-range rows are all cut into whole bins of at least
4 positions (no splitVector layout: L = n bs) take it: a read adds its partial overlaps to the
first and last bins it touches and +1 / -1 to a difference array of the full bins between, so
a row is O(n bins) of work (C2: 200 bins of 20 bp).  Each case checks it against the CPU
oracle (validity; integer numerators exact through binsum; means within 1e-12 relative) and
bit for bit against the general kernel on the same plan (kernel="general")."""

import numpy as np
import pytest

from tests.test_gpu_random import CHROM_LEN, check, make_reads, single_rows

pytestmark = pytest.mark.gpu


def plans(reads, seqlen, rows, bins, strand_filter=None, heavy_threshold=-1, kernel="bins"):
    from recoup_amd.engine import Plan, ReadSet
    from tests import oracle_rows
    rs = ReadSet(*reads, seqlen, device=0, strand_filter=strand_filter)
    fast = Plan(rs, rows, bins, kernel=kernel, heavy_threshold=heavy_threshold)
    general = Plan(rs, rows, bins, kernel="general", heavy_threshold=heavy_threshold)
    assert general.info["pileup_kernel"] == 0
    r_fast, r_gen = fast.run(binsum=True), general.run(binsum=True)
    ix = oracle_rows.index_for(reads, seqlen, strand_filter)
    exp = oracle_rows.profile(oracle_rows.row_coverage(ix, rows), bins)
    return r_fast, r_gen, fast.info["pileup_kernel"], exp


def same(a, b):
    np.testing.assert_array_equal(a[1], b[1])
    assert np.array_equal(a[0].view(np.uint64), b[0].view(np.uint64))  # bit-identical doubles
    np.testing.assert_array_equal(a[2], b[2])                             # int64 numerators


@pytest.mark.parametrize("width,n_bins", [(4000, 200), (2000, 500), (2000, 1), (4096, 512), (1000, 40), (999, 37)])
def test_bins_kernel(gpu, width, n_bins):
    """C2's 20-bp bins, 4-bp bins, one bin per row, the 512-bin maximum, odd widths; NULL rows
    (negative index, past the chromosome end)."""
    from recoup_amd.engine import Bins
    rng = np.random.default_rng(700 + n_bins)
    reads = make_reads(rng, 80_000, star_frac=0.1)
    rows = single_rows(rng, 333, width, edge=True)
    rows.start[1], rows.end[1] = 1, width  # (a start at 0 would shorten the row: an R-RNG layout)
    fast, gen, kind, exp = plans(reads, CHROM_LEN, rows, Bins([("whole", n_bins)]))
    assert kind == 4
    check(fast, exp)
    same(fast, gen)


@pytest.mark.parametrize("strand_filter", [None, "+"])
def test_bins_stranded_rows(gpu, strand_filter):
    """ignore.strand = FALSE: up to three candidate streams per row, both row orientations."""
    from recoup_amd.engine import Bins, RowTable
    rng = np.random.default_rng(731)
    reads = make_reads(rng, 70_000, star_frac=0.25)
    r0 = single_rows(rng, 260, 4000)
    rows = RowTable(r0.seg_off, r0.chrom, r0.start, r0.end, r0.strand, ignore_strand=False)
    fast, gen, kind, exp = plans(reads, CHROM_LEN, rows, Bins([("whole", 100)]), strand_filter)
    assert kind == 4
    check(fast, exp)
    same(fast, gen)


@pytest.mark.parametrize("width", [1, 180])
def test_bins_uniform_width_reads_and_heavy_rows(gpu, width):
    """Reads of one width (the start-only stream), deep hot spots piled by the heavy slice
    kernel (low threshold), the linear scale factor."""
    from recoup_amd.engine import Bins
    rng = np.random.default_rng(743 + width)
    reads = make_reads(rng, 150_000, widths=(width, width), star_frac=0.2)
    rows = single_rows(rng, 300, 4000)
    for heavy in (-1, 64):
        bins = Bins([("whole", 200)], scale=0.37)
        fast, gen, kind, exp = plans(reads, CHROM_LEN, rows, bins, heavy_threshold=heavy)
        assert kind == 4
        check(fast, exp)
        same(fast, gen)


def test_bins_flank_slice(gpu):
    """One binned part that is a slice of the row (binCoverageMatrix(where = "upstream")),
    forward and reversed rows."""
    from recoup_amd.engine import Bins
    rng = np.random.default_rng(757)
    reads = make_reads(rng, 90_000, widths=(30, 300))
    rows = single_rows(rng, 280, 3000)
    for where, nb in (("upstream", 50), ("downstream", 25), ("center", 100)):
        bins = Bins([(where, nb)], flank=(1000, 1000))
        fast, gen, kind, exp = plans(reads, CHROM_LEN, rows, bins)
        assert kind == 4
        check(fast, exp)
        same(fast, gen)


def test_bins_kernel_choice(gpu):
    """AUTO takes the bin-difference kernel for one binned part of uniform bins >= 4 positions;
    2-bp bins (C4), R-RNG layouts, medians, per-base and multi-part plans keep their kernels."""
    from recoup_amd.engine import Bins, Plan, ReadSet
    rng = np.random.default_rng(761)
    reads = make_reads(rng, 20_000)
    rs = ReadSet(*reads, CHROM_LEN, device=0)
    rows = single_rows(rng, 50, 4000)
    assert Plan(rs, rows, Bins([("whole", 200)])).info["pileup_kernel"] == 4
    assert Plan(rs, rows, Bins([("whole", 500)])).info["pileup_kernel"] == 4   # bs 8
    assert Plan(rs, rows, Bins([("whole", 1000)])).info["pileup_kernel"] == 0  # > 512 bins
    assert Plan(rs, rows, Bins([("whole", 2000)])).info["pileup_kernel"] == 0  # bs 2 (general below 36k rows)
    assert Plan(rs, rows, Bins([("whole", 150)])).info["pileup_kernel"] == 0   # R-RNG layout
    assert Plan(rs, rows, Bins([("whole", 200)], stat="median")).info["pileup_kernel"] == 0
    assert Plan(rs, rows, Bins([("whole", 0, 4000)])).info["pileup_kernel"] == 1
    parts = Bins([("upstream", 50), ("center", 100), ("downstream", 50)], flank=(1000, 1000))
    assert Plan(rs, rows, parts).info["pileup_kernel"] != 4
    assert Plan(rs, rows, Bins([("whole", 200)]), kernel="general").info["pileup_kernel"] == 0


def test_bins_repeated_executions(gpu):
    """One plan executed three times (heavy slots cleared by the next execution's locate) gives
    the same bits each time."""
    from recoup_amd.engine import Bins, Plan, ReadSet
    rng = np.random.default_rng(769)
    reads = make_reads(rng, 120_000, widths=(100, 200))
    rs = ReadSet(*reads, CHROM_LEN, device=0)
    rows = single_rows(rng, 200, 4000)
    plan = Plan(rs, rows, Bins([("whole", 200)]), kernel="bins", heavy_threshold=64)
    first = plan.run()
    for _ in range(2):
        again = plan.run()
        assert np.array_equal(again[0].view(np.uint64), first[0].view(np.uint64))
