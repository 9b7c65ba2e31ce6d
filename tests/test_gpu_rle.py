"""Profiles of the reference's own coverage object -- a list of Rle (R/coverage.R:171-173) --
through rcp_profile_rle (R/profile.R:100-212 on a stored or sliced $coverage,
R/recoup.R:126-135, R/util.R:209-210).  coverageRef -> to_list(rle=True) -> profileMatrix must
equal the fused device pass (DeviceCoverage) bit for bit for integer Rle and the oracle on
random cases: uniform and R-RNG bins, interpolation (spline / neighborhood / "inear"),
median, per-base flanks, NULL rows, numeric (normalised) Rle, dense vectors, slices."""
import numpy as np
import pytest

import recoup_amd as ra
from recoup_amd.engine import Bins, profile_rle
from tests import helpers, oracle_rows
from tests.test_gpu_random import CHROM_LEN, make_reads, single_rows

pytestmark = pytest.mark.gpu
FLANK = (2000, 2000)


def _c1_inputs(region, flank, keep=None):
    """coverageRef of test.input over test.genome twice: one sample list keeps the
    DeviceCoverage, the other the materialised list of Rle (as a saved recoup object has it).
    keep: number of reads kept of sample 2 (unequal library sizes)."""
    from tests.golden import c1_cases
    from tests.test_gpu_api import _input
    d = c1_cases.load_inputs()
    G = c1_cases.genome(d)
    genome = ra.GRanges(G["chrom"], G["start"], G["end"], G["strand"], names=G["names"])

    def inputs():
        inp = _input({"d": d})
        if keep is not None:
            inp[1]["ranges"] = inp[1]["ranges"][np.arange(keep)]
        return inp
    inp_dev = ra.coverageRef(inputs(), genome, region, flank)
    inp_rle = ra.coverageRef(inputs(), genome, region, flank)
    for s in inp_rle:
        s["coverage"] = s["coverage"].to_list(rle=True)
    return genome, inp_dev, inp_rle


def _bits(a, b):
    assert a.shape == b.shape
    assert np.array_equal(np.ascontiguousarray(a).view(np.uint64), np.ascontiguousarray(b).view(np.uint64))


@pytest.mark.parametrize("region,bp", [("tss", {"flankBinSize": 0, "regionBinSize": 200}),
                                       ("tss", {"flankBinSize": 0, "regionBinSize": 0}),
                                       ("tss", {"flankBinSize": 0, "regionBinSize": 150}),
                                       ("genebody", {"flankBinSize": 50, "regionBinSize": 150}),
                                       ("genebody", {"flankBinSize": 0, "regionBinSize": 150, "sumStat": "median"}),
                                       ("genebody", {"flankBinSize": 50, "regionBinSize": 150, "interpolation": "spline"})])
def test_rle_list_equals_device_pass(gpu, region, bp):
    genome, inp_dev, inp_rle = _c1_inputs(region, FLANK)
    ra.profileMatrix(inp_dev, FLANK, bp)
    ra.profileMatrix(inp_rle, FLANK, bp)
    for a, b in zip(inp_dev, inp_rle):
        if bp.get("interpolation") == "spline" or bp.get("sumStat") == "median":
            np.testing.assert_allclose(b["profile"], a["profile"], rtol=1e-12, atol=0)
        else:
            _bits(np.asarray(a["profile"]), np.asarray(b["profile"]))
        assert a["profile"].rownames == b["profile"].rownames


def test_sliced_coverage(gpu):
    """sliceObj subsets the stored coverage list (R/util.R:209-210); its profile is the same
    rows of the full profile."""
    genome, inp_dev, inp_rle = _c1_inputs("genebody", FLANK)
    bp = {"flankBinSize": 50, "regionBinSize": 150}
    ra.profileMatrix(inp_dev, FLANK, bp)
    idx = [3, 0, 17, 42, 42, 99]
    for s in inp_rle:
        cov = s["coverage"]
        s["coverage"] = ra.CoverageList([cov[i] for i in idx], [cov.names[i] for i in idx])
    ra.profileMatrix(inp_rle, FLANK, bp)
    for a, b in zip(inp_dev, inp_rle):
        _bits(np.asarray(a["profile"])[idx], np.asarray(b["profile"]))


def test_numeric_rle_after_linear_normalisation(gpu):
    """normalize = "linear" multiplies the stored coverage (a numeric Rle afterwards)."""
    genome, inp_dev, inp_rle = _c1_inputs("tss", FLANK, keep=37_000)
    f = ra.calcLinearFactors(inp_dev)
    assert (f != 1).any()
    ra.normalizeLinear(inp_dev)
    ra.normalizeLinear(inp_rle)
    for bp in ({"flankBinSize": 0, "regionBinSize": 200}, {"flankBinSize": 0, "regionBinSize": 150, "sumStat": "median"}):
        a = ra.profileMatrix([dict(s, profile=None) for s in inp_dev], FLANK, bp)
        b = ra.profileMatrix([dict(s, profile=None) for s in inp_rle], FLANK, bp)
        for x, y in zip(a, b):
            np.testing.assert_allclose(y["profile"], x["profile"], rtol=1e-13, atol=1e-300)


@pytest.mark.parametrize("stat", ["mean", "median"])
@pytest.mark.parametrize("interp", ["auto", "spline", "neighborhood", "linear"])
def test_random_rle_vs_oracle(gpu, stat, interp):
    """Random rows of mixed lengths (some shorter than the bins: interpolation; R-RNG layouts;
    NULL rows) as integer Rle, dense vectors and a numeric Rle: vs the oracle's splitVector."""
    rng = np.random.default_rng(7 + len(interp) + (stat == "median"))
    reads = make_reads(rng, 60_000)
    R = 180
    rows = single_rows(rng, R, 1000)
    rows.end[:] = rows.start + rng.integers(40, 3000, R)  # mixed lengths
    rows.end[::11] = rows.start[::11] + 30                # short rows (< 100 bins)
    ix = oracle_rows.index_for(reads, CHROM_LEN)
    cov = oracle_rows.row_coverage(ix, rows)
    cov[5] = None
    bins = Bins([("whole", 100)], stat=stat, interp=interp)
    exp, ev = oracle_rows.profile(cov, bins)
    rle = [None if x is None else ra.Rle(*_runs(x)) for x in cov]
    for inp in (rle, cov):
        mat, valid = profile_rle(inp, bins)
        np.testing.assert_array_equal(valid, ev.astype(bool))
        np.testing.assert_allclose(mat, exp, rtol=1e-9, atol=1e-12, equal_nan=True)
    # numeric Rle: x * 0.37 as doubles; the oracle bins the same doubles
    covd = [None if x is None else x * 0.37 for x in cov]
    rled = [None if x is None else ra.Rle(*_runs(x)) for x in covd]
    exp_d = np.vstack([np.zeros(100) if x is None else
                       _row(x, 100, interp, stat) for x in covd])
    mat, _ = profile_rle(rled, bins)
    np.testing.assert_allclose(mat, exp_d, rtol=1e-12, atol=1e-12, equal_nan=True)


def _row(x, n, interp, stat):
    from oracle import oracle as o
    r = o.split_vector(x, n, interp=interp, stat=stat)
    return np.resize(r, n)  # rbind recycles a short row ("inear")


def _runs(x):
    x = np.asarray(x)
    if x.size == 0:
        return x[:0], np.zeros(0, np.int64)
    cut = np.flatnonzero(x[1:] != x[:-1]) + 1
    st = np.concatenate([[0], cut])
    return x[st], np.diff(np.concatenate([st, [x.size]]))


def test_flanks_per_base_and_errors(gpu):
    """Per-base flanks + binned centre (profile.R:58-77) and the reference's errors."""
    rng = np.random.default_rng(3)
    reads = make_reads(rng, 50_000)
    rows = single_rows(rng, 60, 6000)
    ix = oracle_rows.index_for(reads, CHROM_LEN)
    cov = oracle_rows.row_coverage(ix, rows)
    bins = helpers.unequal_bins((1000, 1000), 0, 150)
    exp, ev = oracle_rows.profile(cov, bins)
    mat, valid = profile_rle([None if x is None else ra.Rle(*_runs(x)) for x in cov], bins)
    np.testing.assert_allclose(mat, exp, rtol=1e-12, atol=0)
    # a per-base part whose width differs from the slice: refused like the device path
    with pytest.raises(ra.UnsupportedError):
        profile_rle(cov, Bins([("whole", 0, 5999)]))
    # neighborhood of fewer than 4 values: R raises an error
    with pytest.raises(ra.SemanticError):
        profile_rle([np.arange(3, dtype=np.int32)], Bins([("whole", 4)], interp="neighborhood"))


@pytest.mark.parametrize("seed,widths", [(0, (5, 300)), (1, (5, 300)), (2, (150, 150))])
def test_coverage_rle_runs_across_sub_chunk_seams(gpu, seed, widths):
    """rcp_coverage_rle counts each row's runs inside the coverage pileup (a wave per sub-chunk
    of the row's positions) plus the seams between sub-chunks: rows shorter than, equal to and
    many times one wave chunk (1023 / 2047 / 4095 positions), flat rows (no reads: one run),
    deep hot spots and NULL rows give the oracle's runs exactly; a NULL row keeps no runs.
    Reads of one width (150) take the start-only stream."""
    from recoup_amd.engine import ReadSet, RowTable, coverage_rle_host
    rng = np.random.default_rng(100 + seed)
    reads = make_reads(rng, 80_000, widths=widths)
    gap = ~((reads[0] == 0) & (reads[2] >= 100_000) & (reads[1] <= 110_000))
    reads = tuple(x[gap] for x in reads)
    lens = np.array([1, 2, 63, 64, 1023, 1024, 1025, 2046, 2047, 2048, 2049, 4095, 4096, 4097, 8191, 12_000,
                     30_000, 65_537], np.int64)
    R = 120
    w = np.concatenate([lens, rng.integers(1, 9000, R - len(lens))])
    rng.shuffle(w)
    chrom = rng.integers(0, 2, R).astype(np.int32)
    start = np.array([rng.integers(1, CHROM_LEN[c] - x + 1) for c, x in zip(chrom, w)], np.int64)
    start[0], start[1] = -50, 0                     # negative index -> NULL; 0 -> dropped index
    start[2] = CHROM_LEN[chrom[2]] - w[2] // 2 + 1  # runs past the chromosome -> NULL
    chrom[3], start[3], w[3] = 0, 101_000, 5000     # no reads there: one run of 0
    strand = rng.integers(0, 3, R).astype(np.int8)
    rows = RowTable.from_ranges(chrom, start, start + w - 1, strand)
    ix = oracle_rows.index_for(reads, CHROM_LEN)
    cov = oracle_rows.row_coverage(ix, rows)
    rs = ReadSet(*reads, CHROM_LEN, device=0)
    run_off, values, lengths, valid = coverage_rle_host(rs, rows)
    assert len(run_off) == R + 1 and run_off[0] == 0
    for r in range(R):
        a, b = run_off[r], run_off[r + 1]
        if cov[r] is None:
            assert not valid[r] and a == b
            continue
        assert valid[r]
        v, ln = _runs(cov[r])
        np.testing.assert_array_equal(values[a:b], v)
        np.testing.assert_array_equal(lengths[a:b], ln)


@pytest.mark.parametrize("devices", [None, (0, 0), (0, 0, 0)], ids=["one", "shards2", "shards3"])
def test_profile_of_device_runs(gpu, devices):
    """rcp_profile_cov: the profile of a calcCoverage result from the runs the handle keeps on the
    device(s) -- one device, or shards whose blocks are in (chromosome, start) order, not the
    caller's (rows placed back) -- bit-equal to rcp_profile_rle of the same runs copied to the
    host and uploaded again: uniform and R-RNG bins, interpolated rows (flank / centre / flank
    parts of unequal rows), per-base parts, median, NULL rows."""
    from recoup_amd.engine import ReadSet, RowTable, Shards, coverage_rle_kept, profile_rle_arrays
    from tests.test_gpu_rows import rna_rows
    rng = np.random.default_rng(404)
    reads = make_reads(rng, 200_000)
    r0 = single_rows(rng, 900, 2000, edge=True)
    r0.start[1], r0.end[1] = 1, 2000  # (a start at 0 shortens its row: not a per-base row of 2000)
    perm = rng.permutation(900)
    single = RowTable.from_ranges(r0.chrom[perm], r0.start[perm], r0.end[perm], r0.strand[perm])
    cases = [(single, Bins([("whole", 200)])), (single, Bins([("whole", 300)])),
             (single, Bins([("whole", 200)], stat="median")), (single, Bins([("whole", 0, 2000)])),
             (rna_rows(rng, 200), Bins([("upstream", 50), ("center", 500), ("downstream", 50)], flank=(2000, 2000))),
             (rna_rows(rng, 200), Bins([("upstream", 0, 2000), ("center", 300), ("downstream", 0, 2000)],
                                       flank=(2000, 2000)))]
    rs = ReadSet(*reads, CHROM_LEN, device=0)
    for rows, bins in cases:
        if devices is None:
            kept = coverage_rle_kept(rs, rows)
        else:
            kept = Shards(*reads, CHROM_LEN, rows, list(devices)).coverage_rle_kept()
        run_off, values, lengths, valid = kept.copy()
        m, v = kept.profile(bins)
        ref, rv = profile_rle_arrays(run_off, lengths, values, (valid == 0).astype(np.uint8), bins, 0)
        np.testing.assert_array_equal(v, rv)
        assert np.array_equal(np.asarray(m).view(np.uint64), np.asarray(ref).view(np.uint64)), (rows.n_rows, bins.n_cols)
        kept.close()
