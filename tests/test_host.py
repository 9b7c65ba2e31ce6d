"""Host logic of the package (no GPU): GRanges construction, the region-window verbs of
R/ranges.R:67-100, the profileMatrix column-part selection (R/profile.R:1-98) and the
coverageRnaRef row table (R/coverage.R:79-124), checked against the oracle's independent
restatement and the reference's documented semantics."""
import os

import numpy as np
import pytest

import recoup_amd as ra
from recoup_amd import api
from oracle import oracle as o
from tests.golden import c1_cases


@pytest.fixture(scope="module")
def c1():
    d = c1_cases.load_inputs()
    return d, c1_cases.genome(d), c1_cases.exons(d)


def _genome(G):
    return ra.GRanges(G["chrom"], G["start"], G["end"], G["strand"], names=G["names"])


def test_granges_basics():
    g = ra.GRanges(["chr2", "chr1", "chr2"], [10, 20, 30], width=[5, 1, 10], strand=["+", "-", "*"],
                   seqlengths={"chr1": 100})
    assert g.seqlevels == ["chr2", "chr1"]
    np.testing.assert_array_equal(g.end, [14, 20, 39])
    np.testing.assert_array_equal(g.strand, [0, 1, 2])
    np.testing.assert_array_equal(g.seqlengths, [-1, 100])
    np.testing.assert_array_equal(g.codes_in(["chr1", "chr3"]), [-1, 0, -1])
    assert len(g.keep_strand("-")) == 1
    sub = g[np.array([True, False, True])]
    np.testing.assert_array_equal(sub.start, [10, 30])
    with pytest.raises(ValueError):
        ra.GRanges(["chr1"], [1], [2], strand=["x"])


@pytest.mark.parametrize("region", ["tss", "tes", "genebody", "custom"])
@pytest.mark.parametrize("flank", [(2000, 2000), (500, 1500), (0, 1000)])
def test_regional_ranges_match_oracle(c1, region, flank):
    _, G, _ = c1
    got = ra.getRegionalRanges(_genome(G), region, flank)
    s, e = o.regional_ranges(G["start"], G["end"], G["strand"], region, flank)
    np.testing.assert_array_equal(got.start, s)
    np.testing.assert_array_equal(got.end, e)


def test_point_regions_use_promoters():
    """custom regions of width 1 (peak summits, config C4) -> promoters (ranges.R:81-83)."""
    g = ra.GRanges(["c"] * 2, [100, 200], [100, 200], ["+", "-"])
    r = ra.getRegionalRanges(g, "custom", (1000, 1000))
    np.testing.assert_array_equal(r.start, [-900, -799])
    np.testing.assert_array_equal(r.end, [1099, 1200])
    assert set(r.width) == {2000}


def test_flanking_ranges(c1):
    _, G, _ = c1
    g = _genome(G)
    up = ra.getFlankingRanges(g, 2000, "upstream")
    s, e = o.promoters(G["start"], G["end"], G["strand"], 2000, 0)
    np.testing.assert_array_equal((up.start, up.end), (s, e))
    dn = ra.getFlankingRanges(g, 700, "downstream")
    s, e = o.flank_end(G["start"], G["end"], G["strand"], 700)
    np.testing.assert_array_equal((dn.start, dn.end), (s, e))


def test_profile_bins_equal_lengths():
    b = api._profile_bins({"regionBinSize": 200, "interpolation": "spline", "sumStat": ["median", "mean"]},
                          (2000, 2000), True, 4000)
    assert b.parts == [("whole", 200)] and b.stat == 1 and b.interp == 0  # interpolation left at "auto"
    b = api._profile_bins({"regionBinSize": 0}, (2000, 2000), True, 4000)
    assert b.parts == [("whole", 0, 4000)] and b.n_cols == 4000


def test_profile_bins_unequal_lengths():
    b = api._profile_bins({"regionBinSize": 150, "flankBinSize": 50}, (2000, 2000), False, 0)
    assert b.parts == [("upstream", 50), ("center", 150), ("downstream", 50)]
    b = api._profile_bins({"regionBinSize": 100, "flankBinSize": 25}, (500, 1500), False, 0)
    # round(2 * 25 * 0.25) = round(12.5) = 12 (R rounds half to even), round(37.5) = 38
    assert b.parts == [("upstream", 12), ("center", 100), ("downstream", 38)]
    b = api._profile_bins({"regionBinSize": 100, "flankBinSize": 0}, (300, 0), False, 0)
    assert b.parts == [("upstream", 0, 300), ("center", 100)] and b.n_cols == 400


def test_rna_row_table(c1):
    d, G, E = c1
    gl = ra.GRangesList(ra.GRanges(E["chrom"], E["start"], E["end"], E["strand"]), E["seg_off"], E["names"])
    levels = ["chr12"]
    rows = api._rna_rows(gl, _genome(G), (2000, 2000), levels, True)
    assert rows.n_rows == len(G["start"])
    n_ex = np.diff(E["seg_off"])
    np.testing.assert_array_equal(np.diff(rows.seg_off), n_ex + 2)
    ls, le = o.promoters(G["start"], G["end"], G["strand"], 2000, 0)
    rs, re_ = o.flank_end(G["start"], G["end"], G["strand"], 2000)
    first, last = rows.seg_off[:-1], rows.seg_off[1:] - 1
    np.testing.assert_array_equal(rows.start[first], ls)
    np.testing.assert_array_equal(rows.end[last], re_)
    assert set(rows.seg_group[first]) == {0} and set(rows.seg_group[last]) == {2}
    # flank[1] == 0 -> 1 bp flanks on both sides (the reference tests flank[1] for the right one too)
    rows0 = api._rna_rows(gl, _genome(G), (0, 2000), levels, True)
    w = rows0.end - rows0.start + 1
    assert set(w[rows0.seg_off[:-1]]) == {1} and set(w[rows0.seg_off[1:] - 1]) == {1}


def test_linear_factors():
    s = [{"ranges": ra.GRanges(["c"] * n, np.arange(1, n + 1), width=10)} for n in (100, 50, 200)]
    np.testing.assert_allclose(ra.calcLinearFactors(s), [0.5, 1.0, 0.25])
    np.testing.assert_allclose(ra.calcLinearFactors(s, {"normalize": "sampleto", "sampleTo": 25}),
                               [0.25, 0.5, 0.125])
    with pytest.raises(ra.SemanticError):
        ra.calcLinearFactors([{"ranges": None}])


# ----------------------------------------------------------------------------- R RNG (product)
def test_product_rng_known_answers():
    """The library's own R RNG (rcp_rng_*) against R's published set.seed(42) outputs."""
    np.testing.assert_array_equal(ra.RRng(42).runif(3), [0.9148060434963554, 0.9370754132978618, 0.2861395347863436])
    assert list(ra.RRng(42).sample_sorted(10, 3)) == [1, 5, 10]
    assert list(ra.RRng(42, "Rounding").sample_sorted(10, 3)) == [3, 9, 10]
    with pytest.raises(ra.SemanticError):
        ra.RRng(1).sample_sorted(5, 6)


def test_product_rng_matches_oracle_sequence():
    """Successive sort(sample(n, k)) calls continue one RNG stream, as lapply() does after a
    single set.seed (R/ranges.R:40-44)."""
    g = ra.RRng(7)
    o.set_seed(7)
    for n, k in [(50000, 1000), (1234, 1234), (99, 3)]:
        np.testing.assert_array_equal(g.sample_sorted(n, k), np.sort(o.sample_int(n, k)))


def _r_unif_index(u_stream, dn):
    """R_unif_index (Rejection): rbits(ceil(log2 n)) until below n, 16 bits per unif_rand."""
    bits = int(np.ceil(np.log2(dn)))
    while True:
        v = 0
        for _ in range(0, bits + 1, 16):
            v = 65536 * v + int(np.floor(next(u_stream) * 65536))
        v &= (1 << bits) - 1
        if v < dn:
            return v


def test_product_rng_hash_variant():
    """n > 1e7, k <= n/2: sample.int's .Internal(sample2()) draws indices until k distinct."""
    n, k = 20_000_001, 50
    o.set_seed(11)
    u = iter(o.runif(5000))
    seen = []
    while len(seen) < k:
        v = _r_unif_index(u, n) + 1
        if v not in seen:
            seen.append(v)
    np.testing.assert_array_equal(ra.RRng(11).sample_sorted(n, k), np.sort(seen))


def test_preprocess_sampleto_on_bam_fixtures():
    bams = [os.path.join(os.path.dirname(__file__), "golden", "bam", f)
            for f in ("WT_H4K20me1_50kr.bam", "Set8KO_H4K20me1_50kr.bam")]
    inp = [{"id": "a", "file": bams[0]}, {"id": "b", "file": bams[1]}]
    inp = ra.preprocessRanges(inp, {"normalize": "sampleto", "sampleTo": 10000, "spliceAction": "keep"})
    o.set_seed(42)
    for s, b in zip(inp, bams):
        full = ra.readBam(b)
        idx = np.sort(o.sample_int(len(full), 10000)) - 1
        assert len(s["ranges"]) == 10000
        np.testing.assert_array_equal(s["ranges"].start, full.start[idx])
        np.testing.assert_array_equal(s["ranges"].strand, full.strand[idx])
    ds = ra.preprocessRanges([{"id": "a", "file": bams[0]}, {"id": "b", "file": bams[1]}],
                             {"normalize": "downsample"})
    assert [len(s["ranges"]) for s in ds] == [50000, 50000]


def test_product_rng_matches_independent_python_restatement():
    """The library's R RNG (recoup_amd/csrc/rcp_rng.h) against tests/rrng.py (pure Python, written
    from R's RNG.c / random.c, independent of both C copies): sort(sample(n, k)) streams continued
    across calls, both sample.kind values, and the n > 1e7 hash variant."""
    from tests.rrng import RRng
    for kind in ("Rejection", "Rounding"):
        for seed in (42, 3, 99991):
            g, py = ra.RRng(seed, kind), RRng(seed, kind)
            for n, k in [(50_000, 700), (1234, 1234), (99, 3), (70_000, 5)]:
                np.testing.assert_array_equal(g.sample_sorted(n, k), np.sort(py.sample_int(n, k)))
    g, py = ra.RRng(11), RRng(11)
    np.testing.assert_array_equal(g.sample_sorted(20_000_001, 50), np.sort(py.sample_int(20_000_001, 50)))


def test_reciprocal_division_is_correctly_rounded(tmp_path):
    """rcp_div_rn (recoup_amd/csrc/rcp_divrn.h), the kernels' bin-mean division RN(x / width)
    through RN(1 / width) and one FMA correction, equals IEEE division: every numerator below
    2^18 over every width 1..600, and 2M random (numerator < 2^32, width < 2^20, scale) triples."""
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = str(tmp_path / "div_rn_check")
    subprocess.check_call(["gcc", "-O2", "-ffp-contract=off", "-I", os.path.join(root, "recoup_amd", "csrc"), "-o",
                           exe, os.path.join(root, "tests", "native", "div_rn_check.c"), "-lm"])
    r = subprocess.run([exe, "18", "600", "2000000"], capture_output=True, text=True)
    assert r.returncode == 0 and r.stdout.strip() == "0", r.stdout + r.stderr


def test_packed_transfer_encoders(tmp_path):
    """The host encoders of the packed transfers (recoup_amd/csrc/rcp_pack.h, rcp_stage.cpp): strand
    codes four to a byte (every byte value in every position; codes outside 0..2 -> 3) and blocks of
    int32 as a base + 16-bit offsets (decoded back exactly; refused exactly when the span is 2^16 or
    more)."""
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = str(tmp_path / "pack_check")
    subprocess.check_call(["gcc", "-O2", "-I", os.path.join(root, "recoup_amd", "csrc"), "-o", exe,
                           os.path.join(root, "tests", "native", "pack_check.c")])
    r = subprocess.run([exe], capture_output=True, text=True)
    assert r.returncode == 0 and r.stdout.strip() == "0", r.stdout + r.stderr
