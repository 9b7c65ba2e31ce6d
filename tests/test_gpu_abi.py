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
