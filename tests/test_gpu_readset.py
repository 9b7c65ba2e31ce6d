"""Readset input forms (rcp_readset_create, splitBySeqname R/util.R:1-13): reads handed over in
any order vs coordinate-sorted (a sorted BAM's readGAlignments, R/ranges.R:111-132: the merged
layout then skips its radix sort and the stranded one sorts on the stream id alone), and the
seqnames given as the runs of GRanges' Rle instead of one code per read.  Every form must give
the same stream index and bit-identical profiles, checked against the oracle."""
import numpy as np
import pytest

from tests import oracle_rows
from tests.test_gpu_random import CHROM_LEN, check, make_reads, single_rows

pytestmark = pytest.mark.gpu


def _sorted(reads, rng, shuffle_ties=True):
    """(chrom, start) order; equal starts in random order (any order is a valid BAM order)."""
    chrom, start, end, strand = reads
    tie = rng.random(len(start))
    o = np.lexsort((tie, start, chrom))
    return tuple(x[o] for x in reads)


def _runs(chrom):
    """run values / lengths of an integer vector (S4Vectors::Rle)."""
    brk = np.flatnonzero(np.diff(chrom)) + 1
    starts = np.concatenate([[0], brk])
    lengths = np.diff(np.concatenate([starts, [len(chrom)]]))
    return chrom[starts].astype(np.int32), lengths.astype(np.int64)


def _profile(reads, rows, bins, **kw):
    from recoup_amd.engine import Plan, ReadSet
    rs = ReadSet(*reads, CHROM_LEN, device=0, strand_filter=kw.pop("strand_filter", None))
    return rs, Plan(rs, rows, bins, **kw).run()


@pytest.mark.parametrize("ignore_strand", [True, False])
def test_sorted_input_same_index_and_profile(gpu, ignore_strand):
    from recoup_amd.engine import Bins, RowTable
    rng = np.random.default_rng(7)
    reads = make_reads(rng, 150_000, star_frac=0.1)
    rows = single_rows(rng, 300, 2000)
    if not ignore_strand:
        rows = RowTable.from_ranges(rows.chrom, rows.start, rows.end, rows.strand, ignore_strand=False)
    bins = Bins([("whole", 100)])
    rs_u, got_u = _profile(reads, rows, bins)
    rs_s, got_s = _profile(_sorted(reads, rng), rows, bins)
    np.testing.assert_array_equal(rs_u.stream_off, rs_s.stream_off)
    np.testing.assert_array_equal(got_u[1], got_s[1])
    np.testing.assert_array_equal(got_u[0].view(np.uint64), got_s[0].view(np.uint64))
    ix = oracle_rows.index_for(reads, CHROM_LEN)
    exp = oracle_rows.profile(oracle_rows.row_coverage(ix, rows), bins)
    check(got_s, exp)


def test_sorted_input_heavy_rows_and_filter(gpu):
    """Sorted input through the heavy path and a strand filter (dropped reads sort last)."""
    from recoup_amd.engine import Bins
    rng = np.random.default_rng(8)
    reads = _sorted(make_reads(rng, 120_000), rng)
    rows = single_rows(rng, 120, 3000)
    bins = Bins([("whole", 150)])
    for sf in (None, "+"):
        rs, got = _profile(reads, rows, bins, strand_filter=sf, heavy_threshold=16)
        ix = oracle_rows.index_for(reads, CHROM_LEN, sf)
        check(got, oracle_rows.profile(oracle_rows.row_coverage(ix, rows), bins))


def test_seqnames_runs(gpu):
    """chrom as (runValue, runLength): host arrays and device arrays, sorted and unsorted
    (an unsorted read order has many short runs)."""
    import torch
    from recoup_amd.engine import Bins, ReadSet
    rng = np.random.default_rng(9)
    reads = make_reads(rng, 100_000, star_frac=0.05)
    rows = single_rows(rng, 200, 1500)
    bins = Bins([("whole", 75)])
    _, ref = _profile(reads, rows, bins)
    for rd in (reads, _sorted(reads, rng)):
        runs = _runs(rd[0])
        assert runs[1].sum() == len(rd[0])
        _, got = _profile((runs,) + tuple(rd[1:]), rows, bins)
        np.testing.assert_array_equal(got[1], ref[1])
        np.testing.assert_array_equal(got[0].view(np.uint64), ref[0].view(np.uint64))
        dev = [torch.as_tensor(x, device="cuda:0") for x in rd[1:]]
        rs = ReadSet(runs, *dev, CHROM_LEN, device=0)
        from recoup_amd.engine import Plan
        got = Plan(rs, rows, bins).run()
        np.testing.assert_array_equal(got[0].view(np.uint64), ref[0].view(np.uint64))


def test_seqnames_runs_errors(gpu):
    from recoup_amd import _lib
    from recoup_amd.engine import ReadSet
    rng = np.random.default_rng(10)
    chrom, start, end, strand = make_reads(rng, 1000)
    with pytest.raises(_lib.RcpError, match="cover"):
        ReadSet((np.array([0, 1], np.int32), np.array([500, 400], np.int64)), start, end, strand, CHROM_LEN)
    with pytest.raises(_lib.RcpError, match="length"):
        ReadSet((np.array([0, 1], np.int32), np.array([1000, 0], np.int64)), start, end, strand, CHROM_LEN)
    # a run code outside the seqlevels drops its reads, as an unknown per-read code does
    rs = ReadSet((np.array([0, 9], np.int32), np.array([600, 400], np.int64)), start, end, strand, CHROM_LEN)
    assert rs.n == 600


@pytest.mark.parametrize("sort", [False, True])
def test_width_runs(gpu, sort):
    """end as the runs of width(x) (IRanges holds start and width): end = start + width - 1 is
    formed on the GPU.  Fixed-length reads (one run), mixed lengths (many runs), zero-width
    reads, seqnames runs together with width runs, host and device starts: the same profile bit
    for bit as the per-read ends, and the oracle's."""
    import torch
    from recoup_amd.engine import Bins, Plan, ReadSet
    rng = np.random.default_rng(19)
    chrom, start, _, strand = make_reads(rng, 60_000)
    for width in (np.full(len(start), 180, np.int32),                                  # one run
                  np.repeat(rng.integers(0, 300, 600), 100).astype(np.int32)):          # 600 runs, zeros
        end = (start.astype(np.int64) + width - 1).astype(np.int32)
        reads = (chrom, start, end, strand)
        if sort:
            o = np.lexsort((start, chrom))
            reads = tuple(x[o] for x in reads)
            width = width[o]
        rows = single_rows(rng, 200, 2000)
        bins = Bins([("whole", 1000)])
        _, ref = _profile(reads, rows, bins)
        exp = oracle_rows.profile(oracle_rows.row_coverage(oracle_rows.index_for(reads, CHROM_LEN), rows), bins)
        check(ref, exp)
        wr = _runs(width)
        assert wr[1].sum() == len(width)
        for ch in (reads[0], _runs(reads[0])):
            _, got = _profile((ch, reads[1], wr, reads[3]), rows, bins)
            np.testing.assert_array_equal(got[1], ref[1])
            np.testing.assert_array_equal(got[0].view(np.uint64), ref[0].view(np.uint64))
        dev = [torch.as_tensor(x, device="cuda:0") for x in (reads[0], reads[1], reads[3])]
        rs = ReadSet(dev[0], dev[1], wr, dev[2], CHROM_LEN, device=0)
        got = Plan(rs, rows, bins).run()
        np.testing.assert_array_equal(got[0].view(np.uint64), ref[0].view(np.uint64))


def test_width_runs_errors(gpu):
    from recoup_amd import _lib
    from recoup_amd.engine import ReadSet
    rng = np.random.default_rng(20)
    chrom, start, end, strand = make_reads(rng, 1000)
    with pytest.raises(_lib.RcpError, match="cover"):
        ReadSet(chrom, start, (np.array([50, 60], np.int32), np.array([500, 400], np.int64)), strand, CHROM_LEN)
    with pytest.raises(_lib.RcpError, match="length"):
        ReadSet(chrom, start, (np.array([50, 60], np.int32), np.array([1000, 0], np.int64)), strand, CHROM_LEN)
    with pytest.raises(_lib.RcpError, match="width"):
        ReadSet(chrom, start, (np.array([50, -1], np.int32), np.array([500, 500], np.int64)), strand, CHROM_LEN)

    # IRanges' ends fit int32: a width run pushing start + width - 1 past 2^31 - 1 is refused
    # (not wrapped to a negative end)
    big = start.copy()
    big[7] = 2 ** 31 - 100
    with pytest.raises(_lib.UnsupportedError, match="2\\^31"):
        ReadSet(chrom, big, (np.array([180], np.int32), np.array([1000], np.int64)), strand, CHROM_LEN)
    ok = ReadSet(chrom, big, (np.array([100], np.int32), np.array([1000], np.int64)), strand, CHROM_LEN)
    assert ok.n == 1000
