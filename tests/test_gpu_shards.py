"""One sample's reads split over several GPUs for one row table (rcp_shards_*, rcp_profile_rle_multi).

The reference parallelises calcCoverage over regions and binCoverageMatrix over rows with
cmclapply (R/coverage.R:147-154, R/profile.R:198-199, R/util.R:364-382).  rcp_shards_create cuts
the rows into one contiguous block per device and gives each device ONLY the reads its block's
regions can overlap (uploaded in slices, counted, redistributed device to device).  The box has
one GPU, so the devices are (0, 0) / (0, 0, 0): every code path of the split runs, with the
"peer" copies inside one device.  Every result must be bit-identical to the single-device path,
and each device must hold exactly the reads its block's regions overlap (uniform read widths:
the candidate ranges are exactly the overlapping reads)."""
import numpy as np
import pytest

from tests.test_gpu_random import CHROM_LEN, make_reads, single_rows
from tests.test_gpu_rows import rna_rows

pytestmark = pytest.mark.gpu


def overlapping(reads, rows, r0, r1, strand_filter=None):
    """Indices of the reads that overlap any range of rows [r0, r1) (findOverlaps, any strand
    compatible with the range when the table is stranded)."""
    chrom, start, end, strand = reads
    keep = np.ones(len(start), bool) if strand_filter is None else strand == {"+": 0, "-": 1}[strand_filter]
    hit = np.zeros(len(start), bool)
    for j in range(int(rows.seg_off[r0]), int(rows.seg_off[r1])):
        s, e = max(int(rows.start[j]), 1), int(rows.end[j])
        if e < s:
            continue
        m = keep & (chrom == rows.chrom[j]) & (start <= e) & (end >= s)
        if not rows.ignore_strand and rows.strand[j] != 2:
            m &= (strand == rows.strand[j]) | (strand == 2)
        hit |= m
    return np.flatnonzero(hit)


def block_order(rows, order):
    """The table with its rows in the shards' order (rcp_shards_rows): block b is rows
    split[b] .. split[b + 1] - 1 of it."""
    from recoup_amd.engine import RowTable
    order = np.asarray(order)
    idx = np.concatenate([np.arange(rows.seg_off[r], rows.seg_off[r + 1]) for r in order]) if len(order) else \
        np.zeros(0, np.int64)
    seg_off = np.concatenate([[0], np.cumsum(np.diff(rows.seg_off)[order])]).astype(np.int64)
    return RowTable(seg_off, rows.chrom[idx], rows.start[idx], rows.end[idx], rows.strand[idx],
                    seg_group=None if rows.seg_group is None else rows.seg_group[idx],
                    group_is_list=rows.group_is_list, ignore_strand=rows.ignore_strand)


def check_order(sh, rows):
    """The shards' row order is a permutation of the table in (chromosome, start) order (the
    chromosome of a row's first range, its lowest start)."""
    order = sh.order()
    assert np.array_equal(np.sort(order), np.arange(rows.n_rows))
    first = rows.seg_off[:-1]
    lo = np.minimum.reduceat(rows.start, first) if len(rows.start) else np.zeros(0)
    key = np.stack([rows.chrom[first][order], lo[order]], 1)
    assert all(tuple(key[i]) <= tuple(key[i + 1]) for i in range(len(key) - 1))
    return block_order(rows, order)


def same_bits(a, b):
    assert a.shape == b.shape
    assert np.array_equal(np.ascontiguousarray(a).view(np.uint64), np.ascontiguousarray(b).view(np.uint64))


def one_device(reads, rows, bins, strand_filter=None, seqlen=CHROM_LEN):
    from recoup_amd.engine import ReadSet, coverage_rle_host, profile_host
    rs = ReadSet(*reads, seqlen, device=0, strand_filter=strand_filter)
    out = np.zeros((bins.n_cols, rows.n_rows), np.float64)
    valid = np.zeros(max(rows.n_rows, 1), np.uint8)
    profile_host(rs, rows, bins, out, valid)
    return (out.T, valid[:rows.n_rows].astype(bool)), coverage_rle_host(rs, rows)


@pytest.mark.parametrize("n_dev", [2, 3])
@pytest.mark.parametrize("table", ["sorted", "chrom_blocks", "shuffled"])
def test_shards_single_range_rows(gpu, n_dev, table):
    """TSS-like windows (binned and per-base profiles, coverage Rle lists): bit-equal to one
    device; each device holds exactly the reads its block's windows overlap.  The blocks are cut
    in (chromosome, start) order whatever the table's order -- position-sorted, chromosomes in
    another order (a few runs of rows per block: copied run by run), shuffled (rows scattered on
    the host) -- so the devices hold the same reads as for the sorted table."""
    from recoup_amd.engine import Bins, RowTable, Shards
    rng = np.random.default_rng(50 + n_dev)
    reads = make_reads(rng, 120_000, widths=(150, 150))
    r0 = single_rows(rng, 500, 2000, edge=True)
    r0.start[1], r0.end[1] = 1, 2000  # (a start at 0 shortens its row: not a per-base row of 2000)
    by_pos = np.lexsort((r0.start, r0.chrom))
    order = {"sorted": by_pos, "chrom_blocks": np.lexsort((r0.start, -r0.chrom)),
             "shuffled": rng.permutation(500)}[table]
    rows = RowTable.from_ranges(r0.chrom[order], r0.start[order], r0.end[order], r0.strand[order])
    sh = Shards(*reads, CHROM_LEN, rows, [0] * n_dev)
    split, held = sh.info()
    assert split[0] == 0 and split[-1] == rows.n_rows and np.all(np.diff(split) > 0)
    brows = check_order(sh, rows)
    for b in range(n_dev):
        assert held[b] == len(overlapping(reads, brows, split[b], split[b + 1]))
    assert held.sum() < 0.8 * n_dev * len(reads[1])  # not replicas
    if table != "sorted":
        s_rows = RowTable.from_ranges(r0.chrom[by_pos], r0.start[by_pos], r0.end[by_pos], r0.strand[by_pos])
        _, held_sorted = Shards(*reads, CHROM_LEN, s_rows, [0] * n_dev).info()
        assert held.sum() <= 1.1 * held_sorted.sum()
    for bins in (Bins([("whole", 1000)]), Bins([("whole", 0, 2000)]), Bins([("whole", 150)])):
        (m1, v1), _ = one_device(reads, rows, bins)
        m, v = sh.profile(bins)
        np.testing.assert_array_equal(v, v1)
        same_bits(m, m1)
    _, cov1 = one_device(reads, rows, Bins([("whole", 100)]))
    cov = sh.coverage_rle()
    for a, b in zip(cov, cov1):
        np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("stranded,strand_filter", [(False, None), (True, None), (True, "-")])
def test_shards_rna_rows(gpu, stranded, strand_filter):
    """coverageRnaRef rows (flank | exon list | flank), strand-split tables and a strand filter:
    the strand-split layout is what the slices index and the blocks rebuild."""
    from recoup_amd.engine import Bins, Shards
    rng = np.random.default_rng(70 + stranded)
    reads = make_reads(rng, 150_000, widths=(60, 60), star_frac=0.2)
    rows = rna_rows(rng, 240, ignore_strand=not stranded)
    sh = Shards(*reads, CHROM_LEN, rows, [0, 0, 0], strand_filter=strand_filter)
    split, held = sh.info()
    brows = check_order(sh, rows)
    for b in range(3):
        assert held[b] == len(overlapping(reads, brows, split[b], split[b + 1], strand_filter))
    bins = Bins([("upstream", 50), ("center", 500), ("downstream", 50)], flank=(2000, 2000), scale=0.73)
    (m1, v1), cov1 = one_device(reads, rows, bins, strand_filter)
    m, v = sh.profile(bins)
    np.testing.assert_array_equal(v, v1)
    same_bits(m, m1)
    for a, b in zip(sh.coverage_rle(), cov1):
        np.testing.assert_array_equal(a, b)


def test_shards_general_widths_heavy_rows_and_na_seqlengths(gpu):
    """Reads of many widths (candidate ranges wider than the overlaps: prefix max of ends), hot
    peaks that take the heavy slice path, NA seqlengths (a region past the hits' last end is
    NULL): bit-equal to one device, and each device holds at least its overlapping reads."""
    from recoup_amd.engine import Bins, RowTable, Shards
    rng = np.random.default_rng(91)
    chrom, start, end, strand = make_reads(rng, 200_000, widths=(20, 900))
    hot = rng.integers(0, 200_000, 40_000)
    start[hot] = 150_000 + rng.integers(0, 300, hot.size).astype(np.int32)
    chrom[hot] = 0
    end[hot] = start[hot] + 100
    reads = (chrom, start, end, strand)
    r0 = single_rows(rng, 400, 2000)
    c = np.concatenate([r0.chrom, [0, 0]]).astype(np.int32)
    s = np.concatenate([r0.start, [149_500, 380_000]])
    rows = RowTable.from_ranges(c, s, s + 1999, np.concatenate([r0.strand, [0, 1]]).astype(np.int8))
    na = np.array([-1, -1, -1], np.int64)
    sh = Shards(*reads, na, rows, [0, 0])
    split, held = sh.info()
    brows = check_order(sh, rows)
    for b in range(2):
        assert held[b] >= len(overlapping(reads, brows, split[b], split[b + 1]))
    for bins in (Bins([("whole", 1000)]), Bins([("whole", 200)], stat="median")):
        (m1, v1), cov1 = one_device(reads, rows, bins, seqlen=na)
        m, v = sh.profile(bins)
        np.testing.assert_array_equal(v, v1)
        same_bits(m, m1)
    for a, b in zip(sh.coverage_rle(), cov1):
        np.testing.assert_array_equal(a, b)


def test_shards_balance_by_reads(gpu):
    """Blocks balance candidate reads, not rows: a table whose first rows sit on a dense pile
    gets a first block with fewer rows."""
    from recoup_amd.engine import RowTable, Shards
    rng = np.random.default_rng(5)
    n = 200_000
    chrom = np.zeros(n, np.int32)
    start = np.where(rng.random(n) < 0.7, rng.integers(1000, 60_000, n), rng.integers(1000, 390_000, n)).astype(np.int32)
    reads = (chrom, start, (start + 99).astype(np.int32), rng.integers(0, 2, n).astype(np.int8))
    s = np.sort(rng.integers(1000, 380_000, 600))
    rows = RowTable.from_ranges(np.zeros(600, np.int32), s, s + 999, np.zeros(600, np.int8))
    split, held = Shards(*reads, CHROM_LEN, rows, [0, 0]).info()
    assert split[1] < 300  # the dense first part of the table is the heavier half
    assert abs(int(held[0]) - int(held[1])) < 0.35 * held.sum()


def test_shards_one_device_and_empty_blocks(gpu):
    """One device (the whole readset), fewer rows than devices (empty blocks), no reads at all."""
    from recoup_amd.engine import Bins, RowTable, Shards
    rng = np.random.default_rng(3)
    reads = make_reads(rng, 30_000)
    rows = RowTable.from_ranges(np.array([0, 1], np.int32), np.array([1000, 5000]), np.array([2999, 6999]),
                                np.array([0, 1], np.int8))
    bins = Bins([("whole", 100)])
    (m1, v1), cov1 = one_device(reads, rows, bins)
    for devs in ([0], [0, 0, 0, 0]):
        sh = Shards(*reads, CHROM_LEN, rows, devs)
        m, v = sh.profile(bins)
        same_bits(m, m1)
        np.testing.assert_array_equal(v, v1)
        for a, b in zip(sh.coverage_rle(), cov1):
            np.testing.assert_array_equal(a, b)
    empty = tuple(x[:0] for x in reads)
    m, v = Shards(*empty, CHROM_LEN, rows, [0, 0]).profile(bins)
    assert not v.any() and not m.any()


@pytest.mark.parametrize("n_dev", [2, 3])
def test_profile_rle_multi(gpu, n_dev):
    """rcp_profile_rle_multi (a stored $coverage list's rows over several GPUs) bit-equal to
    rcp_profile_rle: integer and numeric Rle, NULL rows, unequal lengths (genebody parts)."""
    from recoup_amd.engine import Bins, ReadSet, coverage_rle_host, profile_rle_arrays
    rng = np.random.default_rng(11 + n_dev)
    reads = make_reads(rng, 100_000)
    rows = rna_rows(rng, 300)
    run_off, values, lengths, valid = coverage_rle_host(ReadSet(*reads, CHROM_LEN, device=0), rows)
    nulls = (1 - valid).astype(np.uint8)
    bins = Bins([("upstream", 50), ("center", 300), ("downstream", 50)], flank=(2000, 2000))
    for vals in (values, values * 0.37):
        one = profile_rle_arrays(run_off, lengths, vals, nulls, bins, device=0)
        multi = profile_rle_arrays(run_off, lengths, vals, nulls, bins, device=[0] * n_dev)
        np.testing.assert_array_equal(multi[1], one[1])
        same_bits(multi[0], one[0])


def test_profile_multi_replicas_balanced_by_counts(gpu):
    """rcp_profile_multi over replicas: blocks follow the counted candidate reads (a hot first
    half takes fewer rows), results bit-equal to one device."""
    from recoup_amd.engine import Bins, ReadSet, RowTable, profile_host, profile_multi
    rng = np.random.default_rng(8)
    n = 150_000
    start = np.where(rng.random(n) < 0.7, rng.integers(1000, 60_000, n), rng.integers(1000, 390_000, n)).astype(np.int32)
    reads = (np.zeros(n, np.int32), start, (start + 99).astype(np.int32), rng.integers(0, 2, n).astype(np.int8))
    s = np.sort(rng.integers(1000, 380_000, 600))
    rows = RowTable.from_ranges(np.zeros(600, np.int32), s, s + 999, np.zeros(600, np.int8))
    bins = Bins([("whole", 100)])
    mat, valid, split = profile_multi(ReadSet.multi(*reads, CHROM_LEN, [0, 0]), rows, bins)
    assert split[1] < 300
    out = np.zeros((bins.n_cols, rows.n_rows))
    v1 = np.zeros(rows.n_rows, np.uint8)
    profile_host(ReadSet(*reads, CHROM_LEN, device=0), rows, bins, out, v1)
    same_bits(mat, out.T)
    np.testing.assert_array_equal(valid, v1.astype(bool))


def test_shards_on_distinct_devices(gpu):
    """Two DIFFERENT GPUs (peer access enabled between them, the reads redistributed by
    hipMemcpyPeerAsync over xGMI, each block's readset and plan on its own device): bit-equal to
    one device.  A one-GPU box cannot run it: skipped by hardware, not passed."""
    from recoup_amd import _lib
    from recoup_amd.engine import Bins, Shards
    if _lib.device_count() < 2:
        pytest.skip("skipped by hardware: one GPU visible (needs 2 for device-to-device copies)")
    rng = np.random.default_rng(202)
    reads = make_reads(rng, 150_000, widths=(150, 150))
    rows = single_rows(rng, 600, 2000)
    for devs in ([0, 1], [1, 0]):
        sh = Shards(*reads, CHROM_LEN, rows, devs)
        split, held = sh.info()
        brows = check_order(sh, rows)
        for b in range(2):
            assert held[b] == len(overlapping(reads, brows, split[b], split[b + 1]))
        for bins in (Bins([("whole", 1000)]), Bins([("whole", 0, 2000)])):
            (m1, v1), cov1 = one_device(reads, rows, bins)
            m, v = sh.profile(bins)
            np.testing.assert_array_equal(v, v1)
            same_bits(m, m1)
        for a, b in zip(sh.coverage_rle(), cov1):
            np.testing.assert_array_equal(a, b)
