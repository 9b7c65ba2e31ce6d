"""The R production path, executed: the .Call shim (r/src/recoup_amd_shim.c) driven with the
exact arguments r/R/rcp.R builds (tests/r_mirror.py, a line-by-line transliteration) through
tests/rmini (an emulation of the R C API; R is not installed), on the reference's own fixture
(C1, data/recoup_test_data.rda) and synthetic multi-chromosome reads.

recoup() with rcp.R dropped in runs coverageRef / coverageRnaRef (R/recoup.R:551-556) ->
calcCoverage's named list of Rle in $coverage -> profileMatrix (:597) -> binCoverageMatrix /
baseCoverageMatrix of that list, plus the forced heatmap binning (:659-714).  Each step below is
checked against the committed golden fixtures (tests/golden/c1_expected.npz) or the CPU oracle:
integer coverage bit-exact, means within 1e-12 relative."""
import os

import numpy as np
import pytest

from oracle import oracle as o
from tests import r_mirror as rm
from tests.golden import c1_cases

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden", "c1_expected.npz")
MEAN_RTOL = 1e-12


@pytest.fixture(scope="module")
def sh(gpu):
    from tests.rmini import rmini
    return rmini.shim()


@pytest.fixture(scope="module")
def c1():
    from recoup_amd.granges import GRanges, GRangesList
    d = c1_cases.load_inputs()
    S, G, E = c1_cases.samples(d), c1_cases.genome(d), c1_cases.exons(d)
    reads = [GRanges(np.full(len(s["start"]), "chr12"), s["start"], s["end"], s["strand"],
                     seqlevels=list(s["seqlevels"]), seqlengths=s["seqlengths"]) for s in S]
    genes = GRanges(G["chrom"], G["start"], G["end"], G["strand"], names=G["names"])
    exons = GRangesList(GRanges(E["chrom"], E["start"], E["end"], E["strand"]), E["seg_off"], names=E["names"])
    idx = [o.Index(np.zeros(len(s["start"]), np.int32), s["start"], s["end"], s["strand"], s["seqlengths"])
           for s in S]
    design = {k: [str(v) for v in d[f"design_{k}"]] for k in ("rownames", "strand", "RNA_status")}
    assert design["rownames"] == [str(n) for n in G["names"]]  # test.design rows = test.genome rows
    return dict(S=S, reads=reads, genes=genes, exons=exons, idx=idx, G=G, E=E, gold=dict(np.load(GOLD)),
                design=design)


def _decode(cov):
    return [None if x is None else np.repeat(x[0], x[1]) for x in cov]


def _assert_cov_equal(got, want):
    assert len(got) == len(want)
    for r, (g, w) in enumerate(zip(got, want)):
        assert (g is None) == (w is None), r
        if g is not None:
            np.testing.assert_array_equal(g, w, err_msg=f"row {r}")


def _oracle_cov(ix, gr, ignore_strand=True):
    m = o.Mask.from_ranges(np.zeros(len(gr), np.int32), gr.start, gr.end, gr.strand)
    return o.coverage(ix, m, ignore_strand, 8)


def _inputs(c1):
    return [dict(id=s["id"], name=s["name"], ranges=g) for s, g in zip(c1["S"], c1["reads"])]


def test_calc_coverage_of_a_split_list(sh, c1):
    """coverageAreaRef's call (R/coverage.R:54-57): calcCoverage(splitBySeqname(reads), mask)."""
    from recoup_amd.granges import getRegionalRanges
    for region in ("tss", "genebody"):
        mask = getRegionalRanges(c1["genes"], region, (2000, 2000))
        for k in range(2):
            got = _decode(rm.calc_coverage(sh, rm.split_by_seqname(c1["reads"][k]), mask))
            _assert_cov_equal(got, _oracle_cov(c1["idx"][k], mask))
    # every readset released (.rcpFree); the coverage lists' device runs live until R collects them
    assert sh.live_handles() == rm.kept_alive(sh)


def _assert_dimnames(m, want, what):
    got = m.dimnames
    assert (got is None) == (want is None), f"{what}: dimnames {got is not None} vs {want is not None}"
    if want is not None:
        assert got[0] == want[0], f"{what}: rownames"
        assert got[1] == want[1], f"{what}: colnames"


def _assert_same_matrix(a, b, what):
    """bit-equal values and identical dimnames (rcp.R's profileMatrix vs the reference's)."""
    np.testing.assert_array_equal(np.asarray(a).view(np.int64), np.asarray(b).view(np.int64), err_msg=what)
    _assert_dimnames(a, b.dimnames, what)


def _design_split_selects_every_row(profile, design_col):
    """R/plot.R:199-204 (and :728-733): split(rownames(x$profile), as.list(d), drop = TRUE), then
    x$profile[splitter[[n]], , drop = FALSE] per design level: rownames must exist, and the
    subsets together hold every row exactly once.  kmeansDesign (R/util.R:181-193) indexes the
    clusters by rownames(design) -- the same names."""
    rn = profile.rownames
    assert rn is not None, "profile without rownames: plot.R:200 splits NULL"
    assert len(set(rn)) == len(rn)
    pos = {n: i for i, n in enumerate(rn)}
    picked = []
    for lvl in sorted(set(design_col)):
        names = [n for n, d in zip(rn, design_col) if d == lvl]
        picked += [pos[n] for n in names]  # profile[names, ] by name
    assert sorted(picked) == list(range(len(rn)))


def test_tss_recoup_path(sh, c1):
    """coverageBaseRef -> $coverage -> profileMatrix (per base, regionBinSize = 0) and the forced
    200-bin heatmap pass (inst/unitTests/test_recoup.R:4-13, R/recoup.R:659-671), with the
    dimnames the reference's rbind leaves: rownames = region names."""
    inp = rm.coverage_ref(sh, _inputs(c1), c1["genes"], "tss", (2000, 2000), {"strand": None, "ignoreStrand": True})
    gold = c1["gold"]
    names = list(c1["G"]["names"])
    for k, x in enumerate(inp):
        valid = np.array([c is not None for c in x["coverage"]])
        np.testing.assert_array_equal(valid, gold[f"tss_valid_s{k}"].astype(bool))
        assert x["coverage"].names == names
    bp = dict(flankBinSize=0, regionBinSize=0)
    inp = rm.profile_matrix(sh, inp, (2000, 2000), bp)
    ref = rm.ref_profile_matrix(sh, [dict(coverage=x["coverage"]) for x in inp], (2000, 2000), bp)
    heat = rm.ref_forced_heatmap(sh, inp, "tss", (2000, 2000), bp)
    for k, x in enumerate(inp):
        np.testing.assert_array_equal(x["profile"], gold[f"tss_base_s{k}"].astype(np.float64))
        _assert_dimnames(x["profile"], o.profile_dimnames(names, (2000, 2000), bp, True), "tss profile")
        _assert_same_matrix(x["profile"], ref[k]["profile"], "tss: rcp.R profileMatrix vs R/profile.R's")
        np.testing.assert_allclose(heat[k], gold[f"tss_heat_s{k}"], rtol=MEAN_RTOL, atol=0)
        _assert_dimnames(heat[k], (names, o.bin_colnames(200, "mean")), "tss heatmap")
        _design_split_selects_every_row(x["profile"], c1["design"]["RNA_status"])
        _design_split_selects_every_row(heat[k], c1["design"]["strand"])
        b150 = rm.bin_coverage_matrix(sh, x["coverage"], 150)  # man/profileMatrix.Rd:32-50
        np.testing.assert_allclose(b150, gold[f"tss150_s{k}"], rtol=MEAN_RTOL, atol=0)
        _assert_dimnames(b150, (names, o.bin_colnames(150, "mean")), "tss 150 bins")


@pytest.mark.parametrize("stat", ["mean", "median"])
def test_genebody_recoup_path(sh, c1, stat):
    """coverageAreaRef -> profileMatrix's unequal-length branch (test_recoup.R:15-26) in one call
    per sample, equal (values and dimnames) to the reference's three binCoverageMatrix calls +
    cbind + rownames<-; the forced heatmap pass of a non-base region stops at R/recoup.R:703."""
    inp = rm.coverage_ref(sh, _inputs(c1), c1["genes"], "genebody", (2000, 2000),
                          {"strand": None, "ignoreStrand": True})
    bp = dict(flankBinSize=50, regionBinSize=150, sumStat=stat, interpolation="auto")
    inp = rm.profile_matrix(sh, inp, (2000, 2000), bp)
    ref = rm.ref_profile_matrix(sh, [dict(coverage=x["coverage"]) for x in inp], (2000, 2000), bp)
    names = list(c1["G"]["names"])
    for k, x in enumerate(inp):
        np.testing.assert_allclose(x["profile"], c1["gold"][f"gb_{stat}_s{k}"], rtol=1e-9 if stat == "median"
                                   else MEAN_RTOL, atol=0)
        _assert_dimnames(x["profile"], o.profile_dimnames(names, (2000, 2000), bp, False), "genebody")
        assert x["profile"].colnames[:2] == ["1." + stat, "2." + stat] and len(x["profile"].colnames) == 250
        _assert_same_matrix(x["profile"], ref[k]["profile"], "genebody: rcp.R profileMatrix vs R/profile.R's")
        _design_split_selects_every_row(x["profile"], c1["design"]["RNA_status"])
    with pytest.raises(NameError, match="forcedBinSize"):
        rm.ref_forced_heatmap(sh, inp, "genebody", (2000, 2000), dict(bp, flankBinSize=0))


def test_genebody_per_base_flanks(sh, c1):
    """flankBinSize = 0 (R/profile.R:58-77): per-base flanks around the binned center; the
    cbind's colnames are "" for the per-base columns."""
    inp = rm.coverage_ref(sh, _inputs(c1), c1["genes"], "genebody", (1000, 500),
                          {"strand": None, "ignoreStrand": True})
    bp = dict(flankBinSize=0, regionBinSize=60, sumStat="mean", interpolation="auto")
    inp = rm.profile_matrix(sh, inp, (1000, 500), bp)
    ref = rm.ref_profile_matrix(sh, [dict(coverage=x["coverage"]) for x in inp], (1000, 500), bp)
    names = list(c1["G"]["names"])
    want = o.profile_matrix([[None if c is None else np.repeat(c[0], c[1]) for c in x["coverage"]] for x in inp],
                            (1000, 500), bp)
    for k, x in enumerate(inp):
        np.testing.assert_allclose(x["profile"], want[k], rtol=MEAN_RTOL, atol=0)
        dn = o.profile_dimnames(names, (1000, 500), bp, False)
        assert dn[1][:1000] == [""] * 1000 and dn[1][1000] == "1.mean" and dn[1][-500:] == [""] * 500
        _assert_dimnames(x["profile"], dn, "genebody per-base flanks")
        _assert_same_matrix(x["profile"], ref[k]["profile"], "per-base flanks: rcp.R vs R/profile.R")


def test_rna_recoup_path(sh, c1):
    """coverageRnaRef (R/coverage.R:79-124) as ONE 3-group pass per sample: its coverage is the
    reference's three calcCoverage passes merged with c(le, ce, ri) (here: three oracle passes),
    and profileMatrix of it matches the golden RNA profile (man/coverageRnaRef.Rd), rows named
    by the exon list (names(genomeRanges), :121)."""
    from recoup_amd.granges import getFlankingRanges
    genes, exons = c1["genes"], c1["exons"]
    inp = rm.coverage_rna_ref(sh, _inputs(c1), exons, genes, (2000, 2000))
    left = getFlankingRanges(genes, 2000, "upstream")
    right = getFlankingRanges(genes, 2000, "downstream")
    E = c1["E"]
    ex = o.Mask(E["seg_off"], np.zeros(len(E["start"]), np.int32), E["start"], E["end"], E["strand"])
    for k, x in enumerate(inp):
        ix = c1["idx"][k]
        want = o.rna_merge(_oracle_cov(ix, left), o.coverage(ix, ex, True, 8), _oracle_cov(ix, right))
        _assert_cov_equal(_decode(x["coverage"]), want)
    bp = dict(flankBinSize=50, regionBinSize=150, interpolation="auto")
    inp = rm.profile_matrix(sh, inp, (2000, 2000), bp)
    ref = rm.ref_profile_matrix(sh, [dict(coverage=x["coverage"]) for x in inp], (2000, 2000), bp)
    for k, x in enumerate(inp):
        np.testing.assert_allclose(x["profile"], c1["gold"][f"rna_s{k}"], rtol=MEAN_RTOL, atol=0)
        _assert_dimnames(x["profile"], o.profile_dimnames(list(E["names"]), (2000, 2000), bp, False), "rna")
        _assert_same_matrix(x["profile"], ref[k]["profile"], "rna: rcp.R profileMatrix vs R/profile.R's")


class _devices:
    """options(recoup.devices = devs) for the duration of a block."""

    def __init__(self, devs):
        self.devs = tuple(devs)

    def __enter__(self):
        self.prev, rm.DEVICES = rm.DEVICES, self.devs

    def __exit__(self, *exc):
        rm.DEVICES = self.prev


def test_profile_from_reads(sh, c1):
    """profileMatrixFromReads: every sample in one rcp_R_profile_reads call, and the rows
    split over two device slots (rcp_R_shards + rcp_R_shards_profile) bit-equal to it."""
    from recoup_amd.granges import getRegionalRanges
    mask = getRegionalRanges(c1["genes"], "tss", (2000, 2000))
    bp = dict(flankBinSize=0, regionBinSize=200)
    one = rm.profile_matrix_from_reads(sh, _inputs(c1), mask, (2000, 2000), bp)
    with _devices((0, 0)):
        two = rm.profile_matrix_from_reads(sh, _inputs(c1), mask, (2000, 2000), bp)
    for k in range(2):
        np.testing.assert_allclose(one[k]["profile"], c1["gold"][f"tss_heat_s{k}"], rtol=MEAN_RTOL, atol=0)
        _assert_dimnames(one[k]["profile"], o.profile_dimnames(list(mask.names), (2000, 2000), bp, True), "reads")
        _assert_same_matrix(two[k]["profile"], one[k]["profile"], "two device slots vs one")
    assert sh.live_handles() == rm.kept_alive(sh)


def _same_coverage(a, b):
    assert a.names == b.names and len(a) == len(b)
    for x, y in zip(a, b):
        assert (x is None) == (y is None)
        if x is not None:
            np.testing.assert_array_equal(x[0], y[0])
            np.testing.assert_array_equal(x[1], y[1])


@pytest.mark.parametrize("devs", [(0, 0), (0, 0, 0)])
def test_recoup_path_on_several_devices(sh, c1, devs):
    """recoup()'s own path with options(recoup.devices = devs): coverageRef (TSS, genebody) and
    coverageRnaRef -> $coverage -> profileMatrix, every step split over the devices (the reads of
    each sample split for its row table, rcp_R_shards; the stored coverage list's rows split,
    rcp_profile_rle_multi) -- bit-equal, coverage and profiles with their dimnames, to one device."""
    genes, exons = c1["genes"], c1["exons"]
    sp = {"strand": None, "ignoreStrand": True}
    runs = [("tss", dict(flankBinSize=0, regionBinSize=0)),
            ("genebody", dict(flankBinSize=50, regionBinSize=150, sumStat="mean", interpolation="auto")),
            ("rna", dict(flankBinSize=50, regionBinSize=150, interpolation="auto"))]
    for region, bp in runs:
        def path():
            if region == "rna":
                inp = rm.coverage_rna_ref(sh, _inputs(c1), exons, genes, (2000, 2000))
            else:
                inp = rm.coverage_ref(sh, _inputs(c1), genes, region, (2000, 2000), sp)
            return rm.profile_matrix(sh, inp, (2000, 2000), bp)
        one = path()
        rm.PATHS.clear()
        with _devices(devs):
            many = path()
        assert "device" in rm.PATHS  # (the shards' coverage handle: parts on each device, in the caller's order)
        for a, b in zip(many, one):
            _same_coverage(a["coverage"], b["coverage"])
            _assert_same_matrix(a["profile"], b["profile"], f"{region}: {len(devs)} devices vs one")
    # calcCoverage straight from a GRanges and from splitBySeqname's list
    from recoup_amd.granges import getRegionalRanges
    mask = getRegionalRanges(genes, "tss", (2000, 2000))
    for inp in (c1["reads"][0], rm.split_by_seqname(c1["reads"][1])):
        one = rm.calc_coverage(sh, inp, mask)
        with _devices(devs):
            _same_coverage(rm.calc_coverage(sh, inp, mask), one)
    # a readset the caller prepared for this mask serves it; for another mask calcCoverage stops
    # instead of returning the prepared mask's coverage under the other mask's names
    with _devices(devs):
        rs = rm.rcp_read_set(sh, c1["reads"][0], rows_of=lambda lv: rm.rcp_rows(mask, lv))
        try:
            _same_coverage(rm.calc_coverage(sh, rs, mask), rm.calc_coverage(sh, c1["reads"][0], mask))
            other = getRegionalRanges(genes, "tss", (1000, 1000))
            with pytest.raises(rm.RStop, match="another mask"):
                rm.calc_coverage(sh, rs, other)
        finally:
            rm.rcp_free(sh, rs)
    assert sh.live_handles() == rm.kept_alive(sh)


def test_split_list_with_merged_seqinfo_and_strands(sh):
    """A list whose elements carry different seqinfo (one chromosome's length NA in one element,
    known in another), reads in any order, the strand filter and ignore.strand = FALSE."""
    from recoup_amd.granges import GRanges
    rng = np.random.default_rng(11)
    lv = ["chr1", "chr2", "chr3"]
    L = {"chr1": 300000, "chr2": 200000, "chr3": 250000}
    parts, codes, starts, ends, strands = {}, [], [], [], []
    for c, name in enumerate(lv):
        n = 4000 + 1000 * c
        st = rng.integers(1, L[name] - 400, n)
        en = st + rng.integers(20, 300, n)
        sd = rng.integers(0, 3, n)
        # chr2's element does not know its own length; chr3's element knows chr2's
        sl = {name: L[name]} if name != "chr2" else {}
        if name == "chr3":
            sl["chr2"] = L["chr2"]
        parts[name] = GRanges(np.full(n, name), st, en, sd, seqlevels=lv if name == "chr3" else [name],
                              seqlengths=sl)
        codes.append(np.full(n, c, np.int32))
        starts.append(st)
        ends.append(en)
        strands.append(sd)
    R = 120
    rc = rng.integers(0, 3, R)
    cen = np.array([rng.integers(3000, L[lv[c]] - 3000) for c in rc])
    rs_ = rng.integers(0, 3, R)
    mask = GRanges(np.array(lv)[rc], cen - 1500, cen + 1499, rs_, seqlevels=lv)
    seqlen = np.array([L[c] for c in lv], np.int64)
    whole = GRanges(np.concatenate([np.full(len(parts[c]), c) for c in lv]), np.concatenate(starts),
                    np.concatenate(ends), np.concatenate(strands), seqlevels=lv, seqlengths=L)
    for strand in (None, "+", "-"):
        if strand is not None:  # strand() of splitBySeqname's plain list stops in the reference
            with pytest.raises(rm.RStop, match="strand"):
                rm.calc_coverage(sh, parts, mask, strand)
        for ign in (True, False):
            # the list (merged seqinfo) without a strand filter; the GRanges with one
            got = _decode(rm.calc_coverage(sh, parts if strand is None else whole, mask, strand, ign))
            ix = o.Index(np.concatenate(codes), np.concatenate(starts), np.concatenate(ends),
                         np.concatenate(strands).astype(np.int8), seqlen,
                         strand_filter=None if strand is None else {"+": 0, "-": 1}[strand])
            m = o.Mask.from_ranges(rc.astype(np.int32), mask.start, mask.end, mask.strand)
            _assert_cov_equal(got, o.coverage(ix, m, ign, 8))


def test_library_errors_unwind_without_leaks(sh, c1):
    """A library error inside rcp_R_coverage (a row table the library rejects) is an R error
    raised after the call returned: the protect stack is reset and the coverage handle, if any,
    is held by a finalizer; the readset stays usable and is released by rcp_R_free."""
    from tests.rmini import rmini
    rs = rm.rcp_read_set(sh, c1["reads"][0])
    rows = rm.rcp_rows(c1["genes"], rs.levels)
    bad = dict(rows, segOff=rows["segOff"][::-1].copy())  # offsets running backwards
    with pytest.raises(rmini.RError, match="recoup_amd"):
        sh.call("rcp_R_coverage", rs.ptr, *rm.rcp_row_args(bad))
    assert sh.unguarded_handles() == 0
    cov = rm.rcp_coverage(sh, rs, rows)
    _assert_cov_equal(_decode(cov), _oracle_cov(c1["idx"][0], c1["genes"]))
    rm.rcp_free(sh, rs)
    sh.run_finalizers()
    assert sh.live_handles() == 0


def test_profiles_from_device_runs(sh, c1):
    """calcCoverage's runs stay on the GPU beside the list it returns (attr "rcpRuns": the handle
    and the addresses of every Rle's vectors); profileMatrix and the forced heatmap pass profile
    them there while the list is unchanged (R/recoup.R:551-597, :659-714), and upload the list's
    own vectors otherwise: an element replaced (the attribute stays, an address differs), a
    linear rescale (a new list, R/recoup.R:559-577), a handle released (save / load).  The same
    bits every way."""
    import copy
    inp = rm.coverage_ref(sh, _inputs(c1), c1["genes"], "tss", (2000, 2000), {"strand": None, "ignoreStrand": True})
    gold = c1["gold"]
    bp = dict(flankBinSize=0, regionBinSize=0)
    rm.PATHS.clear()
    inp = rm.profile_matrix(sh, inp, (2000, 2000), bp)
    heat = rm.ref_forced_heatmap(sh, inp, "tss", (2000, 2000), bp)
    assert rm.PATHS and set(rm.PATHS) == {"device"}, rm.PATHS
    for k, x in enumerate(inp):
        np.testing.assert_array_equal(x["profile"], gold[f"tss_base_s{k}"].astype(np.float64))
        np.testing.assert_allclose(heat[k], gold[f"tss_heat_s{k}"], rtol=MEAN_RTOL, atol=0)
    cov = inp[0]["coverage"]
    dev = rm.bin_coverage_matrix(sh, cov, 200)
    # cov2[[i]] <- Rle(same runs): R keeps the list's attributes, the element is a new object
    i = next(j for j, x in enumerate(cov) if x is not None)
    cov2 = copy.copy(cov)
    cov2[i] = rm.Rle(cov[i][0].copy(), cov[i][1].copy(), sh)
    rm.PATHS.clear()
    up = rm.bin_coverage_matrix(sh, cov2, 200)
    assert rm.PATHS == ["upload"]
    _assert_same_matrix(up, dev, "an element replaced: uploaded")
    # a runValue changed in the copy: its profile differs where the value does
    cov3 = copy.copy(cov)
    cov3[i] = rm.Rle(cov[i][0] + 1, cov[i][1].copy(), sh)
    assert not np.array_equal(rm.bin_coverage_matrix(sh, cov3, 200)[i], dev[i])
    # lapply(cov, function(x) x * f): a new list without the attribute
    scaled = rm.NamedList([None if x is None else rm.Rle(x[0] * 0.5, x[1], sh) for x in cov], cov.names)
    rm.PATHS.clear()
    half = rm.bin_coverage_matrix(sh, scaled, 200)
    assert rm.PATHS == ["upload"]
    np.testing.assert_allclose(half, 0.5 * dev, rtol=1e-15, atol=0)
    # the handle released (what load() of a saved object leaves): uploaded
    sh.call("rcp_R_cov_free", cov.rcp_runs["handle"])
    rm.PATHS.clear()
    _assert_same_matrix(rm.bin_coverage_matrix(sh, cov, 200), dev, "released handle: uploaded")
    assert rm.PATHS == ["upload"]
    # options(recoup.deviceRuns = FALSE): the runs are released at once
    rm.DEVICE_RUNS = False
    try:
        n0 = rm.kept_alive(sh)
        inp2 = rm.coverage_ref(sh, _inputs(c1), c1["genes"], "tss", (2000, 2000), {"strand": None, "ignoreStrand": True})
        assert inp2[0]["coverage"].rcp_runs is None and rm.kept_alive(sh) == n0
    finally:
        rm.DEVICE_RUNS = True
    assert sh.live_handles() == rm.kept_alive(sh)
