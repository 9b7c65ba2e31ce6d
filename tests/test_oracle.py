"""Pinning the CPU oracle (oracle/, test infrastructure) before it is trusted as the checker.

Anchors, in decreasing strength:
  1. R RNG known answers (set.seed / runif / sample, both sample.kind values);
  2. the reference's own fixture data/recoup_test_data.rda (tests/golden/recoup_test_data.npz):
     the sanity numbers of the C1 probe and the committed golden matrices regenerate bit-exactly;
  3. independent pure-numpy restatements of coverageFromRanges (R/coverage.R:176-226) and
     splitVector (R/util.R:15-85) on randomized small inputs, including the NULL rules,
     GRangesList duplicate hits, strand compatibility and the interpolation branches.
R itself is absent from this image, so the oracle is "partially pinned" (DESIGN.md).
"""
import os
import warnings

import numpy as np
import pytest

from oracle import oracle as o
from tests.golden import c1_cases

HERE = os.path.dirname(os.path.abspath(__file__))


# ----------------------------------------------------------------------------- R RNG
def test_runif_known_answer():
    o.set_seed(42)
    np.testing.assert_array_equal(o.runif(3), [0.9148060434963554, 0.9370754132978618, 0.2861395347863436])


def test_sample_known_answers():
    o.set_seed(42)
    assert list(o.sample_int(10, 10, "Rejection")) == [1, 5, 10, 8, 2, 4, 6, 9, 7, 3]
    o.set_seed(42)
    assert list(o.sample_int(10, 10, "Rounding")) == [10, 9, 3, 6, 4, 8, 5, 1, 2, 7]


def test_sample_is_a_permutation_prefix():
    for n in (1, 2, 7, 100, 4001):
        o.set_seed(42)
        s = o.sample_int(n, n)
        assert sorted(s) == list(range(1, n + 1))
    with pytest.raises(ValueError):
        o.sample_int(3, 4)


# ----------------------------------------------------------------------------- C1 anchors
@pytest.fixture(scope="module")
def gold():
    return dict(np.load(os.path.join(HERE, "golden", "c1_expected.npz")))


def test_c1_probe_sanity_numbers(gold):
    """Appendix B: TSS +-2000 per-base over the 100 test genes (61 '+', 39 '-')."""
    d = c1_cases.load_inputs()
    G = c1_cases.genome(d)
    assert (G["strand"] == 0).sum() == 61 and (G["strand"] == 1).sum() == 39
    expect = [(6, 147912, 8, 0.36978), (4, 129624, 7, 0.32406)]
    for k, (zero, total, mx, heat_mean) in enumerate(expect):
        base = gold[f"tss_base_s{k}"]
        assert base.shape == (100, 4000)
        assert int((base.sum(axis=1) == 0).sum()) == zero
        assert int(base.sum()) == total
        assert int(base.max()) == mx
        assert round(float(gold[f"tss_heat_s{k}"].mean()), 5) == heat_mean


def test_c1_genebody_widths():
    G = c1_cases.genome(c1_cases.load_inputs())
    w = G["end"] - G["start"] + 1
    assert (w.min(), w.max(), round(float(np.median(w)))) == (54, 823499, 29594)


def test_c1_fixtures_regenerate(gold):
    """make_fixtures.py --expected is reproducible: the committed matrices are the oracle's."""
    res = c1_cases.compute_all_with_oracle(nthreads=4)
    assert set(res) == set(gold)
    for k in gold:
        np.testing.assert_array_equal(res[k], gold[k], err_msg=k)


def test_c1_heatmap_is_binned_per_base(gold):
    """dif = 0 layout (4000 / 200): each heatmap bin is the mean of 20 consecutive bases."""
    for k in range(2):
        base = gold[f"tss_base_s{k}"].astype(np.float64)
        np.testing.assert_allclose(base.reshape(100, 200, 20).mean(axis=2), gold[f"tss_heat_s{k}"],
                                   rtol=1e-15, atol=0)


# ----------------------------------------------------------------------------- coverage
def _bf_coverage(reads, seqlen, rows, ignore_strand):
    """coverageFromRanges (R/coverage.R:176-226) restated with numpy, one row at a time."""
    rc, rs, re_, rst = reads
    out = []
    for segs in rows:
        chrom0, strand0 = segs[0][0], segs[0][3]
        on = rc == chrom0
        if not on.any():  # splitBySeqname drops empty chromosomes -> "not found" -> NULL
            out.append(None)
            continue
        hits = []
        for (c, s, e, st) in segs:
            if c != chrom0 or e < s:
                continue
            m = on & (rs <= e) & (re_ >= s)
            if not ignore_strand and st != 2:
                m &= (rst == st) | (rst == 2)
            hits.extend(np.nonzero(m)[0].tolist())
        if not hits:
            out.append(None)
            continue
        hits = np.array(hits)
        L = seqlen[chrom0] if seqlen[chrom0] >= 0 else int(re_[hits].max())
        depth = np.zeros(L + 2, dtype=np.int64)
        np.add.at(depth, rs[hits], 1)
        np.add.at(depth, np.minimum(re_[hits], L) + 1, -1)
        depth = np.cumsum(depth)
        idx = np.concatenate([np.arange(s, e + 1) for (_, s, e, _) in segs])
        if (idx > L).any() or ((idx < 0).any() and (idx > 0).any()):
            out.append(None)  # subscript error -> tryCatch -> NULL
            continue
        v = depth[idx[idx != 0]].astype(np.int32)
        out.append(v[::-1].copy() if strand0 == 1 else v)
    return out


def _random_case(rng, n_reads=600, na_seqlen=False):
    seqlen = np.array([4000, 2500, 3000], dtype=np.int64)
    chrom = rng.integers(0, 2, n_reads).astype(np.int32)  # chromosome 2 has no reads
    w = rng.integers(1, 150, n_reads)
    start = (rng.integers(1, seqlen[chrom] - w + 2)).astype(np.int32)
    end = (start + w - 1).astype(np.int32)
    strand = rng.integers(0, 3, n_reads).astype(np.int8)
    if na_seqlen:
        seqlen = seqlen.copy()
        seqlen[1] = -1
    rows = []
    for _ in range(120):
        kind = rng.integers(0, 10)
        c = int(rng.integers(0, 3))
        st = int(rng.integers(0, 3))
        if kind < 6:  # single range, sometimes touching / crossing the ends
            s = int(rng.integers(-20, 4100))
            e = s + int(rng.integers(0, 400))
            rows.append([(c, s, e, st)])
        else:  # GRangesList element: 2-4 ascending exons, shared strand
            k = int(rng.integers(2, 5))
            pos = np.sort(rng.choice(np.arange(1, 3900), size=2 * k, replace=False))
            rows.append([(c, int(pos[2 * j]), int(pos[2 * j + 1]), st) for j in range(k)])
    return (chrom, start, end, strand), seqlen, rows


def _mask(rows):
    off = np.zeros(len(rows) + 1, dtype=np.int64)
    off[1:] = np.cumsum([len(r) for r in rows])
    flat = [s for r in rows for s in r]
    return o.Mask(off, [s[0] for s in flat], [s[1] for s in flat], [s[2] for s in flat], [s[3] for s in flat])


@pytest.mark.parametrize("seed", [0, 1, 2])
@pytest.mark.parametrize("ignore_strand", [True, False])
def test_coverage_matches_numpy_restatement(seed, ignore_strand):
    rng = np.random.default_rng(seed)
    reads, seqlen, rows = _random_case(rng, na_seqlen=(seed == 2))
    ix = o.Index(*reads, seqlen)
    got = o.coverage(ix, _mask(rows), ignore_strand)
    exp = _bf_coverage(reads, seqlen, rows, ignore_strand)
    n_null = 0
    for r, (g, e) in enumerate(zip(got, exp)):
        if e is None:
            assert g is None, r
            n_null += 1
        else:
            assert g is not None, r
            np.testing.assert_array_equal(g, e, err_msg=f"row {r}")
    assert 0 < n_null < len(rows)


def test_coverage_strand_filter():
    """calcCoverage(strand=...) keeps only reads of that strand (R/coverage.R:141-144)."""
    rng = np.random.default_rng(5)
    reads, seqlen, rows = _random_case(rng)
    keep = reads[3] == 1
    filt = tuple(a[keep] for a in reads)
    got = o.coverage(o.Index(*reads, seqlen, strand_filter="-"), _mask(rows))
    exp = _bf_coverage(filt, seqlen, rows, True)
    for g, e in zip(got, exp):
        assert (g is None) == (e is None)
        if e is not None:
            np.testing.assert_array_equal(g, e)


def test_coverage_zero_start_drops_index_zero():
    reads = (np.zeros(2, np.int32), np.array([1, 5], np.int32), np.array([10, 20], np.int32), np.zeros(2, np.int8))
    ix = o.Index(*reads, np.array([100], np.int64))
    cov = o.coverage(ix, o.Mask.from_ranges([0, 0, 0], [0, -1, 95], [9, 9, 101], [0, 0, 0]))
    np.testing.assert_array_equal(cov[0], [1, 1, 1, 1, 2, 2, 2, 2, 2])  # length L - 1
    assert cov[1] is None  # mixed-sign subscript
    assert cov[2] is None  # beyond the sequence length


# ----------------------------------------------------------------------------- splitVector
def _r_mean(x):
    """R's mean.default: long-double sum / n plus the long-double residual correction."""
    x = np.asarray(x, dtype=np.longdouble)
    m = x.sum() / len(x)
    m = m + (x - m).sum() / len(x)
    return float(m)


def _bf_split_vector(x, n, interp, stat, kind):
    x = np.asarray(x, dtype=np.float64)
    L = len(x)
    if L < n:
        mode = interp
        if interp == "auto":
            mode = "neighborhood" if (n - L) / n < 0.2 else "spline"
        if mode == "spline":
            x = np.maximum(o.spline(x, n), 0.0)
        elif mode == "neighborhood":
            y = np.full(n, np.nan)
            y[0:2] = x[0:2]
            y[n - 2:] = x[L - 2:]
            o.set_seed(42)
            pool = np.arange(3, n - 1)
            pick = o.sample_int(len(pool), L - 4, kind) if len(pool) > 1 else o.sample_int(int(pool[0]), L - 4, kind)
            pos = np.sort(pool[pick - 1] if len(pool) > 1 else pick)
            y[pos - 1] = x[2:L - 2]
            na = np.nonzero(np.isnan(y))[0]
            with warnings.catch_warnings():  # all four neighbours NA -> NaN, as mean(na.rm=TRUE)
                warnings.simplefilter("ignore", RuntimeWarning)
                fill = [np.nanmean(y[[z - 2, z - 1, z + 1, z + 2]]) for z in na]
            y[na] = fill
            x = y
        # "linear" (the reference's "inear" typo) leaves x as is
    L = len(x)
    bs = L // n
    dif = L - bs * n
    sizes = np.full(n, bs)
    o.set_seed(42)
    if dif > 0:
        sizes[o.sample_int(n, dif, kind) - 1] += 1
    cuts = np.cumsum(sizes)[:-1]
    out = []
    for b in np.split(x, cuts):
        if len(b) == 0:  # empty factor levels vanish from split()
            continue
        out.append(_r_mean(b) if stat == "mean" else float(np.median(b)))
    return np.array(out)


@pytest.mark.parametrize("kind", ["Rejection", "Rounding"])
@pytest.mark.parametrize("stat", ["mean", "median"])
def test_split_vector_layout(kind, stat):
    rng = np.random.default_rng(11)
    for L, n in [(4000, 200), (4000, 150), (2000, 1000), (29594, 150), (1001, 7), (5, 5), (523, 50)]:
        x = rng.integers(0, 9, L).astype(np.float64)
        got = o.split_vector(x, n, "auto", stat, kind)
        exp = _bf_split_vector(x, n, "auto", stat, kind)
        np.testing.assert_array_equal(got, exp, err_msg=f"L={L} n={n}")


@pytest.mark.parametrize("interp", ["auto", "spline", "neighborhood", "linear"])
def test_split_vector_interpolation(interp):
    rng = np.random.default_rng(3)
    for L, n in [(54, 150), (140, 150), (95, 100), (10, 11), (7, 50)]:
        x = rng.integers(0, 6, L).astype(np.float64)
        got = o.split_vector(x, n, interp, "mean")
        exp = _bf_split_vector(x, n, interp, "mean", "Rejection")
        assert len(got) == len(exp)
        np.testing.assert_allclose(got, exp, rtol=1e-13, atol=1e-13, err_msg=f"{interp} L={L} n={n}")


def test_spline_fmm_reproduces_cubics():
    """fmm end conditions fit cubics through the end points, so cubic data is reproduced exactly."""
    L, n = 37, 150
    t = np.arange(1, L + 1, dtype=np.float64)
    f = lambda u: 0.02 * u ** 3 - 0.5 * u ** 2 + 3 * u + 1  # noqa: E731
    xo = np.linspace(1, L, n)
    np.testing.assert_allclose(o.spline(f(t), n), f(xo), rtol=1e-10, atol=1e-9)


def test_split_vector_neighborhood_too_short_errors():
    with pytest.raises(ValueError):
        o.split_vector(np.ones(3), 4, "neighborhood", "mean")


# ----------------------------------------------------------------------------- R RNG, independent
@pytest.mark.parametrize("kind", ["Rejection", "Rounding"])
def test_rng_matches_independent_python_restatement(kind):
    """The oracle's C R-RNG (rcp_oracle.c) against tests/rrng.py, a pure-Python restatement of
    R's set.seed / MT19937 / unif_rand / sample.int written from R's RNG.c and random.c alone:
    the same draws for many seeds and sizes -- one and two 16-bit chunks per index (n above
    65536), powers of two, whole permutations, and several calls continuing one stream."""
    from tests.rrng import RRng
    for seed in (42, 1, 7, 123456, 2 ** 31 - 1, -5):
        py = RRng(seed, kind)
        o.set_seed(seed)
        np.testing.assert_array_equal(o.runif(5), py.runif(5))
        for n, k in [(10, 10), (200, 37), (4096, 4096), (4097, 150), (65536, 300), (65537, 300),
                     (1_000_003, 500), (3, 1), (1, 1)]:
            np.testing.assert_array_equal(o.sample_int(n, k, kind), py.sample_int(n, k), err_msg=f"{seed} {n} {k}")


def test_split_vector_layout_against_independent_rng():
    """splitVector's enlarged bins (R/util.R:74-80) from the independent RNG: the oracle's bins of
    (L, n) are floor(L / n) + 1 wide exactly on sample(1:n, L %% n) after set.seed(42)."""
    from tests.rrng import RRng
    for L, n in [(4000, 150), (29594, 150), (1001, 7), (523, 50), (2049, 1000)]:
        x = np.arange(L, dtype=np.float64)
        sizes = np.full(n, L // n)
        add = RRng(42).sample_int(n, L - (L // n) * n)
        sizes[np.array(add, dtype=np.int64) - 1] += 1
        cuts = np.concatenate([[0], np.cumsum(sizes)])
        exp = np.array([x[a:b].mean() for a, b in zip(cuts[:-1], cuts[1:])])
        np.testing.assert_allclose(o.split_vector(x, n, "auto", "mean", "Rejection"), exp, rtol=1e-15)
