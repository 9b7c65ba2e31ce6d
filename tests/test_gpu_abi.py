"""The C ABI as an R .Call shim uses it: the one-shot host-pointer entry point
rcp_profile, the coverage + Rle entry points, and the error contract (negative codes, a
message from rcp_last_error, no partial output) on a real device."""
import ctypes
import os

import numpy as np
import pytest
import torch

from recoup_amd import _lib
from recoup_amd.engine import Bins, Plan, RowTable
from tests import helpers

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden", "c1_expected.npz")


@pytest.fixture(scope="module")
def c1(gpu):
    d, S, G, E = helpers.c1()
    return dict(S=S, G=G, rs=[helpers.readset(s) for s in S], gold=dict(np.load(GOLD)))


def _profile(rs, rows, bins):
    """What the shim does: R allocates the R x B double matrix and the logical vector."""
    rd, bd = rows.desc(), bins.desc()
    out = np.full((rows.n_rows, bins.n_cols), np.nan, order="F")  # R column-major
    valid = np.zeros(rows.n_rows, np.uint8)
    rc = _lib.lib().rcp_profile(rs.h, ctypes.byref(rd), ctypes.byref(bd), out.ctypes.data_as(_lib._dp),
                                valid.ctypes.data_as(_lib._u8p))
    return rc, out, valid


def test_rcp_profile_host_buffers(c1):
    rows = helpers.tss_rows(c1["G"])
    for k, rs in enumerate(c1["rs"]):
        rc, out, valid = _profile(rs, rows, Bins([("whole", 200)]))
        assert rc == 0
        np.testing.assert_allclose(out, c1["gold"][f"tss_heat_s{k}"], rtol=1e-12, atol=0)
        np.testing.assert_array_equal(valid, c1["gold"][f"tss_valid_s{k}"])
        rc, out, _ = _profile(rs, rows, Bins([("whole", 0, 4000)]))
        assert rc == 0
        np.testing.assert_array_equal(out, c1["gold"][f"tss_base_s{k}"].astype(np.float64))


def test_rcp_profile_errors_leave_output_untouched(c1):
    rows = helpers.tss_rows(c1["G"])
    # per-base part whose width differs from the rows' length: the library refuses
    rc, out, _ = _profile(c1["rs"][0], rows, Bins([("whole", 0, 3999)]))
    assert rc == -4 and b"width" in _lib.lib().rcp_last_error()
    assert np.isnan(out).all()
    # nine parts: more than RCP_MAX_PARTS
    rc, out, _ = _profile(c1["rs"][0], rows, Bins([("whole", 10)] * 9))
    assert rc == -1 and np.isnan(out).all()


def test_invalid_row_tables(c1):
    rs = c1["rs"][0]
    bad_groups = RowTable(np.array([0, 2]), np.zeros(2, np.int32), np.array([10, 50]), np.array([20, 60]),
                          np.zeros(2, np.int8), seg_group=np.array([1, 0], np.int8))
    with pytest.raises(_lib.RcpError):
        Plan(rs, bad_groups, Bins([("whole", 2)]))
    two_chroms = RowTable(np.array([0, 2]), np.array([0, 1], np.int32), np.array([10, 50]), np.array([20, 60]),
                          np.zeros(2, np.int8), seg_group=np.zeros(2, np.int8),
                          group_is_list=np.array([1, 0, 0, 0], np.uint8))
    with pytest.raises(_lib.UnsupportedError):
        Plan(rs, two_chroms, Bins([("whole", 2)]))


def test_execute_contract(c1):
    rs = c1["rs"][0]
    rows = helpers.tss_rows(c1["G"])
    cov_only = Plan(rs, rows, None)
    with pytest.raises(_lib.RcpError):  # a calcCoverage plan has no columns to execute
        cov_only.execute(torch.empty((1, rows.n_rows), dtype=torch.float64, device="cuda:0"))
    p = Plan(rs, rows, Bins([("whole", 200)]))
    assert _lib.lib().rcp_plan_execute(p.h, None, None, None, None) == -1  # NULL output
    # the padded column stride needs out_ld * (n_cols - 1) + n_rows elements: the unpadded
    # (n_cols, n_rows) shape, a float32 or a host buffer is refused before any launch
    pp = Plan(rs, rows, Bins([("whole", 200)]), out_ld="padded")
    assert pp.out_ld == pp.info["out_ld"] == 112
    for bad in (torch.empty((200, rows.n_rows), dtype=torch.float64, device="cuda:0"),
                torch.empty((200, 112), dtype=torch.float32, device="cuda:0"),
                torch.empty((200, 112), dtype=torch.float64)):
        with pytest.raises(ValueError):
            pp.execute(bad)
    with pytest.raises(ValueError):
        pp.execute(pp.empty_output(), binsum=torch.empty((200, rows.n_rows), dtype=torch.int64, device="cuda:0"))
    np.testing.assert_array_equal(p.validity(), c1["gold"]["tss_valid_s0"].astype(bool))
    np.testing.assert_array_equal(p.row_lengths(), np.full(rows.n_rows, 4000))


def test_readset_info_and_strand_filter(c1):
    from recoup_amd.engine import ReadSet
    s = c1["S"][0]
    chrom = np.zeros(len(s["start"]), np.int32)
    full = ReadSet(chrom, s["start"], s["end"], s["strand"], s["seqlengths"])
    minus = ReadSet(chrom, s["start"], s["end"], s["strand"], s["seqlengths"], strand_filter="-")
    assert full.n == len(s["start"])
    assert minus.n == int((s["strand"] == 1).sum())
    assert full.stream_off[-1] == full.n and full.stream_off[0] == 0
    # reads of an unknown chromosome code or strand code are dropped, not an error
    bad = chrom.copy()
    bad[:10] = 7
    st = s["strand"].copy()
    st[10:20] = 5
    r = ReadSet(bad, s["start"], s["end"], st, s["seqlengths"])
    assert r.n == len(s["start"]) - 20


@pytest.mark.parametrize("n", [13, 1_001, 17_000_003])
def test_strand_codes_cross_pcie(gpu, n):
    """Host strand codes through both upload paths (rcp_stage.h: the direct copy below 4 MB,
    the pinned staging above it): each (chromosome, strand) stream holds exactly the reads of
    that code, and codes outside 0..2 (-1, 3, 5, -128) drop their reads."""
    from recoup_amd.engine import ReadSet
    rng = np.random.default_rng(n)
    codes = np.array([0, 1, 2, 0, 1, 2, 0, 1, 2, -1, 3, 5, -128], np.int8)
    strand = codes[rng.integers(0, len(codes), n)]
    chrom = rng.integers(0, 2, n).astype(np.int32)
    start = rng.integers(1, 1_000_000, n).astype(np.int32)
    end = start + 49
    seql = np.array([2_000_000, 2_000_000], np.int64)
    rs = ReadSet(chrom, start, end, strand, seql)
    keep = (strand >= 0) & (strand <= 2)
    assert rs.n == int(keep.sum())
    so = rs.stream_off
    for c in range(2):
        for q in range(3):
            assert so[3 * c + q + 1] - so[3 * c + q] == int(((chrom == c) & (strand == q)).sum()), (c, q)
    plus = ReadSet(chrom, start, end, strand, seql, strand_filter="+")
    assert plus.n == int((strand == 0).sum())


@pytest.mark.parametrize("n_rows,n_bins", [(20_003, 200), (4_099, 4000)])
def test_rcp_profile_staged_copy(gpu, n_rows, n_bins):
    """rcp_profile's output above the 4 MB direct-copy limit travels through the pinned
    double-buffered stager (64 MB chunks, 4 host threads) from a padded device column stride
    (n_rows rounded up to 16) into R's n_rows x n_cols matrix: bit-equal to the device result."""
    from recoup_amd.engine import ReadSet
    from tests.test_gpu_random import CHROM_LEN, make_reads, single_rows
    rng = np.random.default_rng(n_rows)
    reads = make_reads(rng, 300_000)
    rows = single_rows(rng, n_rows, 4000)
    bins = Bins([("whole", n_bins)])
    rs = ReadSet(*reads, CHROM_LEN, device=0)
    ref, rv = Plan(rs, rows, bins).run()
    rc, out, valid = _profile(rs, rows, bins)
    assert rc == 0 and out.nbytes > (4 << 20)
    assert np.array_equal(out.view(np.uint64), np.asfortranarray(ref).view(np.uint64))
    np.testing.assert_array_equal(valid.astype(bool), rv)


@pytest.mark.parametrize("n_dev,R,nb", [(3, 500, 100), (2, 300, 1000), (4, 3, 40)])
def test_profile_multi_bit_equal(gpu, n_dev, R, nb):
    """rcp_profile_multi (one host thread per device, row blocks copied into the caller's matrix)
    gives the bits of the single-device pass.  The box has one GPU, so the 'devices' are n_dev
    readsets on device 0 driven by n_dev concurrent host threads (R = 3 < 4 devices: an empty
    block)."""
    from recoup_amd.engine import ReadSet, profile_multi
    from tests.test_gpu_random import CHROM_LEN, make_reads, single_rows
    rng = np.random.default_rng(11 + n_dev)
    reads = make_reads(rng, 80_000)
    rows = single_rows(rng, R, 2000, edge=R > 10)
    bins = Bins([("whole", nb)])
    rs = ReadSet(*reads, CHROM_LEN, device=0)
    ref, rvalid = Plan(rs, rows, bins).run()
    multi = ReadSet.multi(*reads, CHROM_LEN, [0] * n_dev)
    mat, valid, split = profile_multi(multi, rows, bins)
    assert split[0] == 0 and split[-1] == R and (np.diff(split) >= 0).all()
    np.testing.assert_array_equal(valid, rvalid)
    assert np.array_equal(mat.view(np.uint64), np.ascontiguousarray(ref).view(np.uint64))
    for r in multi:
        r.close()


def test_coverage_rle_host_one_shot(c1):
    """rcp_coverage_rle (what the R shim binds for calcCoverage): the host Rle list equals the
    device calcCoverage + rcp_rle_encode path, NULL rows included."""
    from recoup_amd.engine import Plan
    rows = helpers.tss_rows(c1["G"])
    L = _lib.lib()
    for rs in c1["rs"]:
        ref = Plan(rs, rows, None).coverage(rle=True)
        rd = rows.desc()
        h = ctypes.c_void_p()
        assert L.rcp_coverage_rle(rs.h, ctypes.byref(rd), ctypes.byref(h)) == 0
        nr, nruns = ctypes.c_int32(), ctypes.c_int64()
        assert L.rcp_cov_info(h, ctypes.byref(nr), ctypes.byref(nruns)) == 0
        assert nr.value == rows.n_rows
        off = np.zeros(nr.value + 1, np.int64)
        vals = np.zeros(max(nruns.value, 1), np.int32)
        lens = np.zeros(max(nruns.value, 1), np.int32)
        valid = np.zeros(nr.value, np.uint8)
        assert L.rcp_cov_copy(h, off.ctypes.data_as(_lib._i64p), vals.ctypes.data_as(_lib._i32p),
                              lens.ctypes.data_as(_lib._i32p), valid.ctypes.data_as(_lib._u8p)) == 0
        assert L.rcp_cov_free(h) == 0
        for r, e in enumerate(ref):
            assert bool(valid[r]) == (e is not None)
            if e is not None:
                np.testing.assert_array_equal(vals[off[r]:off[r + 1]], e[0])
                np.testing.assert_array_equal(lens[off[r]:off[r + 1]], e[1])


@pytest.mark.parametrize("n_samples,inflight,nb", [(4, 2, 100), (5, 3, 1000), (3, 1, 40), (2, 0, 0)])
def test_profile_samples_bit_equal(gpu, n_samples, inflight, nb):
    """rcp_profile_samples (profileMatrix's loop over a recoup input list's samples, passes kept
    `inflight` deep on separate HIP streams, each matrix staged into its own host array) gives
    every sample the bits of its own single pass; nb = 0 is a per-base part."""
    from recoup_amd.engine import ReadSet, profile_samples
    from tests.test_gpu_random import CHROM_LEN, make_reads, single_rows
    rng = np.random.default_rng(40 + n_samples)
    rows = single_rows(rng, 700, 2000, edge=nb > 0)  # (a per-base part needs equal row widths)
    bins = Bins([("whole", nb)]) if nb else Bins([("whole", 0, 2000)])
    rss = [ReadSet(*make_reads(rng, 60_000 + 5_000 * i, star_frac=0.1), CHROM_LEN, device=0)
           for i in range(n_samples)]
    got = profile_samples(rss, rows, bins, inflight=inflight)
    assert len(got) == n_samples
    for rs, (mat, valid) in zip(rss, got):
        ref, rvalid = Plan(rs, rows, bins).run()
        np.testing.assert_array_equal(valid, rvalid)
        assert np.array_equal(mat.view(np.uint64), np.ascontiguousarray(ref).view(np.uint64))


def test_profile_samples_errors(c1):
    from recoup_amd.engine import profile_samples
    rows = helpers.tss_rows(c1["G"])
    with pytest.raises(_lib.RcpError, match="inflight"):
        profile_samples(c1["rs"], rows, Bins([("whole", 20)]), inflight=4)
    assert profile_samples([], rows, Bins([("whole", 20)])) == []


def test_release_pool_then_rebuild(c1):
    """rcp_release_pool returns the library pool's cached device memory; readsets built before
    and after give the same profiles (the pool only recycles memory)."""
    L = _lib.lib()
    rows = helpers.tss_rows(c1["G"])
    bins = Bins([("whole", 200)])
    s = c1["S"][0]
    rs = helpers.readset(s)
    rc, before, vb = _profile(rs, rows, bins)
    assert rc == 0
    del rs
    assert L.rcp_release_pool(0) == 0
    assert L.rcp_release_pool(0) == 0  # nothing cached: still fine
    rs = helpers.readset(s)
    rc, after, va = _profile(rs, rows, bins)
    assert rc == 0
    assert np.array_equal(before.view(np.int64), after.view(np.int64)) and np.array_equal(vb, va)
    assert L.rcp_release_pool(-1) != 0  # a device that does not exist


@pytest.mark.parametrize("n_samples,nb,stranded", [(3, 1000, False), (4, 0, False), (2, 150, True), (1, 40, False)])
def test_profile_reads_pipelined(gpu, n_samples, nb, stranded):
    """rcp_profile_reads (sample k + 1 uploaded while sample k is profiled and copied down) gives
    every sample the bits of its own readset + one-shot profile; reads as runs or per-read ends."""
    from recoup_amd.engine import ReadSet, RowTable, profile_host, profile_reads
    from tests.test_gpu_random import CHROM_LEN, make_reads, single_rows
    rng = np.random.default_rng(140 + n_samples)
    r0 = single_rows(rng, 500, 2000, edge=nb > 0)
    rows = RowTable(r0.seg_off, r0.chrom, r0.start, r0.end, r0.strand, ignore_strand=not stranded)
    bins = Bins([("whole", nb)]) if nb else Bins([("whole", 0, 2000)])
    samples = [make_reads(rng, 50_000 + 7_000 * i, star_frac=0.1, widths=(100, 100) if i % 2 else (20, 400))
               for i in range(n_samples)]
    got = profile_reads(samples, CHROM_LEN, rows, bins)
    for reads, (mat, valid) in zip(samples, got):
        out = np.zeros((bins.n_cols, rows.n_rows))
        v1 = np.zeros(rows.n_rows, np.uint8)
        profile_host(ReadSet(*reads, CHROM_LEN, device=0), rows, bins, out, v1)
        np.testing.assert_array_equal(valid, v1.astype(bool))
        assert np.array_equal(mat.view(np.uint64), np.ascontiguousarray(out.T).view(np.uint64))


def test_profile_rle_row_blocks(gpu):
    """A long Rle list is profiled in row blocks through two streams (runs of one block up while
    another block's rows come down): the same bits as per-row oracle means and as a short list."""
    from recoup_amd.engine import profile_rle_arrays
    rng = np.random.default_rng(99)
    R = 6000  # 2.5 M runs: four row blocks
    lens = rng.integers(1, 4, size=(R, 620)).astype(np.int32)
    L = lens.sum(axis=1)
    keep = L >= 1000
    lens, L = lens[keep], L[keep]
    R = len(L)
    # trim every row to 1000 positions: drop runs past it and shorten the last one
    runs, vals, off = [], [], [0]
    for r in range(R):
        c = np.cumsum(lens[r])
        k = int(np.searchsorted(c, 1000))
        x = lens[r][:k + 1].copy()
        x[-1] -= c[k] - 1000
        runs.append(x)
        vals.append(rng.integers(0, 50, k + 1).astype(np.int32))
        off.append(off[-1] + k + 1)
    lengths, values = np.concatenate(runs), np.concatenate(vals)
    run_off = np.array(off, np.int64)
    nulls = (rng.random(R) < 0.05).astype(np.uint8)
    bins = Bins([("whole", 100)])
    mat, valid = profile_rle_arrays(run_off, lengths, values, nulls, bins)
    assert run_off[-1] > (1 << 21)
    dense = [np.repeat(v, ln) for v, ln in zip(vals, runs)]
    want = np.array([np.zeros(100) if nulls[r] else dense[r].reshape(100, 10).mean(axis=1) for r in range(R)])
    np.testing.assert_array_equal(valid, nulls == 0)
    np.testing.assert_allclose(mat, want, rtol=1e-12, atol=0)
    few = profile_rle_arrays(run_off[:101].copy(), lengths[:run_off[100]], values[:run_off[100]], nulls[:100], bins)
    assert np.array_equal(few[0].view(np.uint64), np.ascontiguousarray(mat[:100]).view(np.uint64))
    # a bad run length in a late block: the blocks check their runs on the device, same message
    from recoup_amd._lib import RcpError
    bad = lengths.copy()
    r_bad = R - 7
    bad[run_off[r_bad] + 1] = 0
    with pytest.raises(RcpError, match=f"row {r_bad}: an Rle run length <= 0"):
        profile_rle_arrays(run_off, bad, values, nulls, bins)


def sorted_sample(rng, n, order=(2, 0, 1), width=100):
    """n reads in (chromosome, start) order with the chromosomes in `order` (a BAM sorted by a
    header whose order is not the seqlevel codes'): the per-read form and the runs form R's
    seqnames(x) / width(x) Rle give (chromosome runs, one width run)."""
    from tests.test_gpu_random import make_reads
    chrom, start, end, strand = make_reads(rng, n, widths=(width, width), star_frac=0.1)
    rank = np.argsort(np.array(order))
    o = np.lexsort((start, rank[chrom]))
    chrom, start, end, strand = chrom[o], start[o], end[o], strand[o]
    cut = np.flatnonzero(np.diff(chrom)) + 1
    cv = chrom[np.r_[0, cut]].astype(np.int32)
    cl = np.diff(np.r_[0, cut, n]).astype(np.int64)
    runs = ((cv, cl), start, (np.array([width], np.int32), np.array([n], np.int64)), strand)
    return (chrom, start, end, strand), runs


def sorted_rows(rng, R, order=(2, 0, 1), ignore_strand=True):
    from recoup_amd.engine import RowTable
    from tests.test_gpu_random import single_rows
    r0 = single_rows(rng, R, 2000)
    rank = np.argsort(np.array(order))
    o = np.lexsort((r0.start, rank[r0.chrom]))
    return RowTable(r0.seg_off, r0.chrom[o], r0.start[o], r0.end[o], r0.strand[o], ignore_strand=ignore_strand)


def one_shot(reads, rows, bins, strand_filter=None):
    from recoup_amd.engine import ReadSet, profile_host
    from tests.test_gpu_random import CHROM_LEN
    out = np.zeros((bins.n_cols, rows.n_rows))
    v1 = np.zeros(rows.n_rows, np.uint8)
    profile_host(ReadSet(*reads, CHROM_LEN, device=0, strand_filter=strand_filter), rows, bins, out, v1)
    return np.ascontiguousarray(out.T), v1.astype(bool)


def traced(capfd, fn):
    import os
    os.environ["RCP_TRACE"] = "1"
    try:
        res = fn()
    finally:
        del os.environ["RCP_TRACE"]
    return res, [ln for ln in capfd.readouterr().err.splitlines() if ln.startswith("[reads]")]


@pytest.mark.parametrize("ignore_strand,strand_filter", [(True, None), (False, None), (False, "-")])
def test_profile_reads_streamed(gpu, capfd, ignore_strand, strand_filter):
    """A coordinate-sorted sample given as runs streams through the GPU in row blocks (each block
    uploads only the slice of reads its rows need while the previous block's rows of the matrix
    come down): the bits of the one-shot readset + profile, on merged and strand-split layouts and
    with a strand filter."""
    from recoup_amd.engine import Bins, profile_reads
    from tests.test_gpu_random import CHROM_LEN
    rng = np.random.default_rng(7 + ignore_strand)
    reads, runs = sorted_sample(rng, 13_000_000)
    rows = sorted_rows(rng, 4000, ignore_strand=ignore_strand)
    bins = Bins([("whole", 100)])
    want = one_shot(reads, rows, bins, strand_filter)
    got, lines = traced(capfd, lambda: profile_reads([runs], CHROM_LEN, rows, bins, strand_filter=strand_filter))
    assert sum("block" in ln for ln in lines) == 3, lines  # 13 M reads: three blocks
    np.testing.assert_array_equal(got[0][1], want[1])
    assert np.array_equal(got[0][0].view(np.uint64), want[0].view(np.uint64))


def test_profile_reads_stream_fallbacks(gpu, capfd):
    """Samples that cannot stream go through whole, with the same bits: a pair of reads out of
    order inside a slice (found on the device after the first slice went up: the sample is redone
    whole), rows in another order than the reads (slices would overlap), a chromosome split over
    two runs.  One call holds all four samples; the first streams."""
    from recoup_amd.engine import Bins, profile_reads
    from tests.test_gpu_random import CHROM_LEN
    rng = np.random.default_rng(21)
    reads, runs = sorted_sample(rng, 4_600_000)
    rows = sorted_rows(rng, 3000)
    bins = Bins([("whole", 0, 2000)])
    n = len(reads[1])
    i = n // 5  # inside the first slice, one chromosome
    while not (reads[1][i] < reads[1][i + 1] and reads[0][i] == reads[0][i + 1]):
        i += 1
    bad_start = reads[1].copy()
    bad_start[[i, i + 1]] = bad_start[[i + 1, i]]
    bad = (runs[0], bad_start, runs[2], runs[3])
    bad_reads = (reads[0], bad_start, bad_start + 99, reads[3])
    cv, cl = runs[0]
    split = ((np.r_[cv[:1], cv]).astype(np.int32), np.r_[cl[:1] // 2, cl[:1] - cl[:1] // 2, cl[1:]].astype(np.int64))
    two_runs = (split, runs[1], runs[2], runs[3])
    got, lines = traced(capfd, lambda: profile_reads([runs, bad, two_runs], CHROM_LEN, rows, bins))
    assert sum("sample 0 block" in ln for ln in lines) == 2, lines
    assert any("sample 1 rows [0, 3000)" in ln for ln in lines), lines
    assert any("sample 2 rows [0, 3000)" in ln for ln in lines), lines
    for (mat, valid), r in zip(got, (reads, bad_reads, reads)):
        m1, v1 = one_shot(r, rows, bins)
        np.testing.assert_array_equal(valid, v1)
        assert np.array_equal(mat.view(np.uint64), m1.view(np.uint64))
    from recoup_amd.engine import RowTable
    perm = rng.permutation(rows.n_rows)
    shuffled = RowTable(rows.seg_off, rows.chrom[perm], rows.start[perm], rows.end[perm], rows.strand[perm])
    got, lines = traced(capfd, lambda: profile_reads([runs], CHROM_LEN, shuffled, bins))
    assert not any("block" in ln for ln in lines), lines
    m1, v1 = one_shot(reads, shuffled, bins)
    assert np.array_equal(got[0][0].view(np.uint64), m1.view(np.uint64))


@pytest.mark.parametrize("n_bins,scale,expand", [(1000, 1.0, True), (1000, 0.37, True), (400, 2.5, True),
                                                 (300, 1.0, False), (5000, 1.0, False)])
def test_matrix_download_as_numerators(gpu, capfd, n_bins, scale, expand):
    """Host matrices travel as uint32 bin numerators when every mean is one (rcp_pack_kernel:
    one-part plans, uniform bins -- power-of-two widths multiply by the reciprocal, others divide --
    NULL rows, a linear scale), the host making each double with the device's operations; R-RNG
    layouts (300 bins of 4000 positions) and interpolated rows (5000 bins) fall back to the doubles.
    Either way bit-equal to the device matrix."""
    from recoup_amd.engine import ReadSet
    from tests.test_gpu_random import CHROM_LEN, make_reads, single_rows
    rng = np.random.default_rng(n_bins)
    reads = make_reads(rng, 300_000)
    rows = single_rows(rng, 6_000, 4000, edge=True)
    bins = Bins([("whole", n_bins)], scale=scale)
    rs = ReadSet(*reads, CHROM_LEN, device=0)
    ref, rv = Plan(rs, rows, bins).run()
    assert not rv.all()  # NULL rows among them
    os.environ["RCP_TRACE"] = "1"
    try:
        rc, out, valid = _profile(rs, rows, bins)
    finally:
        del os.environ["RCP_TRACE"]
    lines = [ln for ln in capfd.readouterr().err.splitlines() if ln.startswith(("[stage] d2h", "[pack]"))]
    assert rc == 0
    assert any("d2h-expand" in ln for ln in lines) == expand, lines
    assert np.array_equal(out.view(np.uint64), np.asfortranarray(ref).view(np.uint64))
    np.testing.assert_array_equal(valid.astype(bool), rv)


@pytest.mark.parametrize("hot_rows", [2, 400], ids=["few_raw_blocks", "many_raw_blocks"])
def test_matrix_download_deep_numerators(gpu, capfd, hot_rows):
    """Bin numerators of 2^16 and more (a deep pile under 40-bp bins) do not fit a block's 16-bit
    offsets: those blocks come down as they are -- block by block when few, the whole chunk when
    many -- fetched by the calling thread on its stream, expanded by the copy threads.  Bit-equal
    to the device matrix either way."""
    from recoup_amd.engine import ReadSet
    from tests.test_gpu_random import CHROM_LEN, make_reads, single_rows
    rng = np.random.default_rng(90 + hot_rows)
    base = make_reads(rng, 300_000)
    k = 9000  # ~3600 deep around chr0:200000 -> bin sums ~1.4e5
    hs = (200_000 + rng.integers(-200, 200, k)).astype(np.int32)
    reads = (np.r_[base[0], np.zeros(k, np.int32)], np.r_[base[1], hs], np.r_[base[2], hs + 179],
             np.r_[base[3], rng.integers(0, 2, k).astype(np.int8)])
    rows = single_rows(rng, 12_000, 4000)
    chrom, start, end, strand = rows.chrom.copy(), rows.start.copy(), rows.end.copy(), rows.strand.copy()
    at = np.arange(100, 100 + hot_rows) if hot_rows < 10 else np.arange(0, 12_000, 12_000 // hot_rows)[:hot_rows]
    chrom[at] = 0
    start[at] = 200_000 - 2000 + rng.integers(-300, 300, len(at))
    end[at] = start[at] + 3999
    rows = RowTable.from_ranges(chrom, start, end, strand)
    bins = Bins([("whole", 100)])
    rs = ReadSet(*reads, CHROM_LEN, device=0)
    ref, rv = Plan(rs, rows, bins).run()
    assert ref.max() * 40 >= 2 ** 16
    os.environ["RCP_TRACE"] = "1"
    try:
        rc, out, valid = _profile(rs, rows, bins)
    finally:
        del os.environ["RCP_TRACE"]
    lines = [ln for ln in capfd.readouterr().err.splitlines() if ln.startswith("[stage] d2h-expand")]
    assert rc == 0 and len(lines) == 1, lines
    n_raw = int(lines[0].split(" raw blocks")[0].rsplit(" ", 1)[1])
    assert n_raw > 0, lines
    assert np.array_equal(out.view(np.uint64), np.asfortranarray(ref).view(np.uint64))
    np.testing.assert_array_equal(valid.astype(bool), rv)


@pytest.mark.parametrize("n_bins,scale,expand", [(1000, 1.0, True), (800, 0.61, True), (300, 1.0, False)])
def test_rle_matrix_download_as_numerators(gpu, capfd, n_bins, scale, expand):
    """recoup()'s Rle path (calcCoverage's list -> rcp_profile_rle): an integer Rle list's profile
    comes down as numerators too (rcp_rle_pack_kernel), R-RNG layouts as doubles; the same bits
    as the fused read profile."""
    from recoup_amd.engine import ReadSet, coverage_rle_host, profile_rle_arrays
    from tests.test_gpu_random import CHROM_LEN, make_reads, single_rows
    rng = np.random.default_rng(7 + n_bins)
    reads = make_reads(rng, 300_000)
    rows = single_rows(rng, 6_000, 4000, edge=True)
    bins = Bins([("whole", n_bins)], scale=scale)
    rs = ReadSet(*reads, CHROM_LEN, device=0)
    ref, rv = Plan(rs, rows, bins).run()
    run_off, values, lengths, valid = coverage_rle_host(rs, rows)
    out = np.full((rows.n_rows, bins.n_cols), np.nan, order="F")
    os.environ["RCP_TRACE"] = "1"
    try:
        profile_rle_arrays(run_off, lengths, values, (valid == 0).astype(np.uint8), bins, 0, out)
    finally:
        del os.environ["RCP_TRACE"]
    lines = [ln for ln in capfd.readouterr().err.splitlines() if ln.startswith(("[stage] d2h", "[pack]"))]
    assert any("d2h-expand" in ln for ln in lines) == expand, lines
    assert np.array_equal(out.view(np.uint64), np.asfortranarray(ref).view(np.uint64))


@pytest.mark.parametrize("sorted_reads", [True, False])
def test_packed_read_uploads(gpu, capfd, sorted_reads):
    """Host read arrays go up packed (rcp_stage.h stage_h2d_i32 / stage_h2d_strand): chromosomes,
    starts and ends as 16-bit offsets from per-1024-read block minima -- blocks spanning 2^16 or
    more (gaps, chromosome changes) raw, chunks with too many such blocks plain (the unsorted
    sample) -- and strand codes four to a byte, codes outside 0..2 still dropping their reads.
    The readset equals one built from the same arrays already on the device: streams, kept reads
    and a profile, bit for bit.  (4.5 M reads with one code each: the codes and strands go up on
    the second H2D lane, beside the starts and ends.)"""
    from recoup_amd.engine import ReadSet
    from tests.test_gpu_random import CHROM_LEN, single_rows
    rng = np.random.default_rng(3 + sorted_reads)
    n = 4_500_000
    codes = np.array([0, 1, 2, 0, 1, 2, -1, 7], np.int8)
    chrom = np.sort(rng.integers(0, 3, n)).astype(np.int32)
    start = np.empty(n, np.int32)
    for c in range(3):
        m = chrom == c
        k = int(m.sum())
        # clustered starts with a few long gaps (raw blocks)
        gaps = rng.geometric(0.05, k).astype(np.int64)
        gaps[rng.random(k) < 2e-4] += 200_000
        start[m] = (1 + np.cumsum(gaps) % (CHROM_LEN[c] - 1000)).astype(np.int32)
    if sorted_reads:
        order = np.lexsort((start, chrom))
        chrom, start = chrom[order], start[order]
    else:
        rng.shuffle(start)
    end = start + rng.integers(0, 300, n).astype(np.int32)
    strand = codes[rng.integers(0, len(codes), n)]
    chrom[rng.integers(0, n, 50)] = 7  # no such chromosome: the read is dropped (one byte, -1, a lane-1 code)
    os.environ["RCP_TRACE"] = "1"
    try:
        host = ReadSet(chrom, start, end, strand, CHROM_LEN, device=0)
    finally:
        del os.environ["RCP_TRACE"]
    lines = [ln for ln in capfd.readouterr().err.splitlines() if "h2d-packed" in ln]
    assert len(lines) == 4, lines  # chrom, start, end, strand
    if not sorted_reads:
        assert any("i32" in ln and " 0 of " not in ln for ln in lines), lines  # plain chunks
    dev = ReadSet(*(torch.from_numpy(a).cuda() for a in (chrom, start, end, strand)), CHROM_LEN, device=0)
    assert host.n == dev.n == int(((strand >= 0) & (strand <= 2) & (chrom < 3)).sum())
    np.testing.assert_array_equal(host.stream_off, dev.stream_off)
    rows = single_rows(rng, 2_000, 3000)
    bins = Bins([("whole", 300)])
    a, b = Plan(host, rows, bins).run(), Plan(dev, rows, bins).run()
    assert np.array_equal(np.ascontiguousarray(a[0]).view(np.uint64), np.ascontiguousarray(b[0]).view(np.uint64))
    np.testing.assert_array_equal(a[1], b[1])


def test_two_lane_upload_many_chromosomes(gpu, capfd):
    """Unsorted reads of a 300-chromosome genome (codes past one byte: the second H2D lane sends
    them as packed int32 blocks, not bytes) beside the starts on the first lane: the readset
    equals one built from the same arrays on the device -- streams, kept reads, a profile."""
    from recoup_amd.engine import ReadSet
    rng = np.random.default_rng(77)
    n_chrom = 300
    lens = rng.integers(200_000, 400_000, n_chrom).astype(np.int64)
    n = 4_500_000
    chrom = rng.integers(0, n_chrom, n).astype(np.int32)
    chrom[rng.integers(0, n, 20)] = n_chrom + 5  # no such chromosome: dropped
    start = (1 + (rng.random(n) * (lens[np.minimum(chrom, n_chrom - 1)] - 1000))).astype(np.int32)
    end = start + rng.integers(0, 300, n).astype(np.int32)
    strand = rng.integers(0, 3, n).astype(np.int8)
    os.environ["RCP_TRACE"] = "1"
    try:
        host = ReadSet(chrom, start, end, strand, lens, device=0)
    finally:
        del os.environ["RCP_TRACE"]
    lines = [ln for ln in capfd.readouterr().err.splitlines() if "h2d-packed" in ln]
    assert not any(" codes " in ln for ln in lines), lines  # > 255 codes: int32 blocks, not bytes
    dev = ReadSet(*(torch.from_numpy(a).cuda() for a in (chrom, start, end, strand)), lens, device=0)
    assert host.n == dev.n == int((chrom < n_chrom).sum())
    np.testing.assert_array_equal(host.stream_off, dev.stream_off)
    rc = rng.integers(0, n_chrom, 1_500).astype(np.int32)
    rs_ = np.array([rng.integers(1, lens[c] - 3000) for c in rc], np.int64)
    rows = RowTable.from_ranges(rc, rs_, rs_ + 2999, rng.integers(0, 2, len(rc)).astype(np.int8))
    bins = Bins([("whole", 300)])
    a, b = Plan(host, rows, bins).run(), Plan(dev, rows, bins).run()
    assert np.array_equal(np.ascontiguousarray(a[0]).view(np.uint64), np.ascontiguousarray(b[0]).view(np.uint64))
    np.testing.assert_array_equal(a[1], b[1])


def test_packed_run_downloads(gpu, capfd):
    """calcCoverage's Rle list comes down packed (rcp_stage.h stage_d2h_i32: per-1024 blocks of
    depths and run lengths as a base + 16-bit offsets, blocks that do not fit -- a zero run of
    2^16 or more positions -- copied as they are): the runs equal the device encoder's, row for
    row."""
    from recoup_amd.engine import ReadSet, RowTable, coverage_rle_host
    from tests.test_gpu_random import CHROM_LEN, make_reads
    rng = np.random.default_rng(5)
    c, st, en, sd = make_reads(rng, 1_500_000, widths=(20, 60), chroms=2)
    # one read on chromosome 3: its 80-kb row is that read and one long zero run
    c, st, en, sd = (np.append(c, 2).astype(np.int32), np.append(st, 1000).astype(np.int32),
                     np.append(en, 1049).astype(np.int32), np.append(sd, 0).astype(np.int8))
    rs = ReadSet(c, st, en, sd, CHROM_LEN, device=0)
    R = 3_000
    rc = rng.integers(0, 2, R)
    rstart = np.array([rng.integers(1, CHROM_LEN[k] - 2000) for k in rc], np.int64)
    rows = RowTable.from_ranges(np.append(rc, 2).astype(np.int32), np.append(rstart, 1000),
                                np.append(rstart + 1999, 80_999), np.zeros(R + 1, np.int8))
    os.environ["RCP_TRACE"] = "1"
    try:
        run_off, values, lengths, valid = coverage_rle_host(rs, rows)
    finally:
        del os.environ["RCP_TRACE"]
    lines = [ln for ln in capfd.readouterr().err.splitlines() if "d2h-packed" in ln]
    assert run_off[-1] >= (1 << 20) and len(lines) == 2, (run_off[-1], lines)
    assert any(" 0 raw blocks" not in ln for ln in lines), lines  # the long zero run
    ref = Plan(rs, rows, None).coverage(rle=True)
    for r, e in enumerate(ref):
        assert bool(valid[r]) == (e is not None)
        if e is not None:
            np.testing.assert_array_equal(values[run_off[r]:run_off[r + 1]], e[0])
            np.testing.assert_array_equal(lengths[run_off[r]:run_off[r + 1]], e[1])
    assert lengths[run_off[R + 1] - 1] == 80_000 - 50  # (the last row: read, then zeros)
