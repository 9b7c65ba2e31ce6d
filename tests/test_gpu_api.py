"""The R-mirroring API on the GPU, written like the reference's own tests
(inst/unitTests/test_recoup.R: TSS per-base, genebody binned; man pages of calcCoverage,
coverageRnaRef and profileMatrix) over the reference's fixture data/recoup_test_data.rda.
Expected values: tests/golden/c1_expected.npz (oracle-made, pinned in tests/test_oracle.py)
and, for coverage lists, the oracle itself."""
import os

import numpy as np
import pytest

import recoup_amd as ra
from oracle import oracle as o
from tests.golden import c1_cases

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden", "c1_expected.npz")
FLANK = (2000, 2000)


@pytest.fixture(scope="module")
def c1(gpu):
    d = c1_cases.load_inputs()
    G = c1_cases.genome(d)
    E = c1_cases.exons(d)
    genome = ra.GRanges(G["chrom"], G["start"], G["end"], G["strand"], names=G["names"])
    exons = ra.GRangesList(ra.GRanges(E["chrom"], E["start"], E["end"], E["strand"]), E["seg_off"], E["names"])
    return dict(d=d, G=G, E=E, genome=genome, exons=exons, gold=dict(np.load(GOLD)))


def _input(c1):
    """test.input: two samples with their reads (recoup_test_data.rda)."""
    out = []
    for s in c1_cases.samples(c1["d"]):
        sl = {lv: int(v) for lv, v in zip(s["seqlevels"], s["seqlengths"]) if v >= 0}
        reads = ra.GRanges(np.full(len(s["start"]), "chr12"), s["start"], s["end"], s["strand"],
                           seqlevels=s["seqlevels"], seqlengths=sl)
        out.append({"id": s["id"], "name": s["name"], "ranges": reads})
    return out


def test_tss_chipseq_per_base(c1):
    """test_recoup.R:4-13 -- region "tss", flank 2000/2000, binParams all zero."""
    inp = ra.coverageRef(_input(c1), c1["genome"], "tss", FLANK)
    inp = ra.profileMatrix(inp, FLANK, {"flankBinSize": 0, "regionBinSize": 0})
    for k, s in enumerate(inp):
        assert s["profile"].shape == (100, 4000)
        np.testing.assert_array_equal(np.asarray(s["profile"]), c1["gold"][f"tss_base_s{k}"].astype(np.float64))
        assert s["profile"].rownames == list(c1["G"]["names"])
        assert s["profile"].colnames is None  # per-base rows: as.numeric(Rle) has no names
        # the forced heatmap pass (recoup.R:659-671): binCoverageMatrix(..., binSize = 200)
        heat = ra.binCoverageMatrix(s["coverage"], binSize=200, stat="mean")
        np.testing.assert_allclose(heat, c1["gold"][f"tss_heat_s{k}"], rtol=1e-12, atol=0)
        assert heat.rownames == list(c1["G"]["names"]) and heat.colnames == o.bin_colnames(200, "mean")
        # a flank slice is mapped over 1:length(cvrg): rbind leaves its rows unnamed
        up = ra.baseCoverageMatrix(s["coverage"], flank=FLANK, where="upstream")
        assert up.rownames is None and up.colnames is None


def test_tss_profile_150_bins(c1):
    """man/profileMatrix.Rd: regionBinSize 150 over 4000 bp -> the set.seed(42) bin layout."""
    inp = ra.coverageRef(_input(c1), c1["genome"], "tss", FLANK)
    inp = ra.profileMatrix(inp, FLANK, {"flankBinSize": 50, "regionBinSize": 150, "sumStat": "mean"})
    for k, s in enumerate(inp):
        np.testing.assert_allclose(s["profile"], c1["gold"][f"tss150_s{k}"], rtol=1e-12, atol=0)


@pytest.mark.parametrize("stat", ["mean", "median"])
def test_genebody_binned(c1, stat):
    """test_recoup.R:15-26 -- region "genebody", flankBinSize 50, regionBinSize 150."""
    inp = ra.coverageRef(_input(c1), c1["genome"], "genebody", FLANK)
    inp = ra.profileMatrix(inp, FLANK, {"flankBinSize": 50, "regionBinSize": 150, "sumStat": stat,
                                        "interpolation": "auto"})
    bp = {"flankBinSize": 50, "regionBinSize": 150, "sumStat": stat}
    for k, s in enumerate(inp):
        assert s["profile"].shape == (100, 250)
        np.testing.assert_allclose(s["profile"], c1["gold"][f"gb_{stat}_s{k}"], rtol=1e-9, atol=1e-12)
        assert (s["profile"].rownames, s["profile"].colnames) == \
            o.profile_dimnames(list(c1["G"]["names"]), FLANK, bp, False)


def test_rna_coverage_profile(c1):
    """man/coverageRnaRef.Rd: exon GRangesList + gene helper ranges."""
    inp = ra.coverageRnaRef(_input(c1), c1["exons"], c1["genome"], FLANK)
    inp = ra.profileMatrix(inp, FLANK, {"flankBinSize": 50, "regionBinSize": 150})
    for k, s in enumerate(inp):
        np.testing.assert_array_equal(s["coverage"].valid(), c1["gold"][f"rna_valid_s{k}"].astype(bool))
        np.testing.assert_allclose(s["profile"], c1["gold"][f"rna_s{k}"], rtol=1e-9, atol=1e-12)
        assert (s["profile"].rownames, s["profile"].colnames) == \
            o.profile_dimnames(list(c1["E"]["names"]), FLANK, {"flankBinSize": 50, "regionBinSize": 150}, False)


def _oracle_index(sample):
    return o.Index(np.zeros(len(sample["start"]), np.int32), sample["start"], sample["end"], sample["strand"],
                   sample["seqlengths"])


def test_calc_coverage_lists(c1):
    """man/calcCoverage.Rd: calcCoverage(reads, genes) and over the exon GRangesList."""
    inp = _input(c1)
    S = c1_cases.samples(c1["d"])
    G, E = c1["G"], c1["E"]
    ix = _oracle_index(S[0])
    cases = [
        (c1["genome"], o.Mask.from_ranges(np.zeros(100, np.int32), G["start"], G["end"], G["strand"]), True),
        (c1["exons"], o.Mask(E["seg_off"], np.zeros(len(E["start"]), np.int32), E["start"], E["end"],
                             E["strand"]), True),
        (c1["genome"], o.Mask.from_ranges(np.zeros(100, np.int32), G["start"], G["end"], G["strand"]), False),
    ]
    for mask, omask, ign in cases:
        got = ra.calcCoverage(inp[0]["ranges"], mask, ignore_strand=ign)
        exp = o.coverage(ix, omask, ign)
        assert len(got) == len(exp)
        for g, e in zip(got, exp):
            assert (g is None) == (e is None)
            if e is not None:
                np.testing.assert_array_equal(g, e)


def test_calc_coverage_strand(c1):
    inp = _input(c1)
    S = c1_cases.samples(c1["d"])
    G = c1["G"]
    ix = o.Index(np.zeros(len(S[1]["start"]), np.int32), S[1]["start"], S[1]["end"], S[1]["strand"],
                 S[1]["seqlengths"], strand_filter="-")
    win = ra.getRegionalRanges(c1["genome"], "tss", FLANK)
    got = ra.calcCoverage(inp[1]["ranges"], win, strand="-")
    exp = o.coverage(ix, o.Mask.from_ranges(np.zeros(100, np.int32), win.start, win.end, win.strand))
    for g, e in zip(got, exp):
        assert (g is None) == (e is None)
        if e is not None:
            np.testing.assert_array_equal(g, e)


def test_device_coverage_lengths_and_list(c1):
    inp = ra.coverageRef(_input(c1), c1["genome"], "genebody", FLANK)
    cv = inp[0]["coverage"]
    lst = cv.to_list()
    np.testing.assert_array_equal(cv.lengths(), lst.lengths())
    assert lst.names == list(c1["G"]["names"])


def test_normalize_linear(c1):
    inp = ra.coverageRef(_input(c1), c1["genome"], "tss", FLANK)
    f = ra.calcLinearFactors(inp)
    inp = ra.normalizeLinear(inp)
    inp = ra.profileMatrix(inp, FLANK, {"flankBinSize": 0, "regionBinSize": 200})
    for k, s in enumerate(inp):
        np.testing.assert_allclose(s["profile"], c1["gold"][f"tss_heat_s{k}"] * f[k], rtol=1e-12, atol=0)


def test_profile_from_host_coverage_list(c1):
    """The reference reuses a stored $coverage (a list of Rle, R/recoup.R:126-135): profileMatrix
    of coverageRef's materialised list equals the fused device pass and the C1 golden matrix."""
    inp = ra.coverageRef(_input(c1), c1["genome"], "tss", FLANK)
    for s in inp:
        s["coverage"] = s["coverage"].to_list(rle=True)
    inp = ra.profileMatrix(inp, FLANK, {"flankBinSize": 0, "regionBinSize": 200})
    for k, s in enumerate(inp):
        np.testing.assert_allclose(s["profile"], c1["gold"][f"tss_heat_s{k}"], rtol=1e-12, atol=0)
        assert s["profile"].rownames == list(c1["G"]["names"])


def test_missing_chromosome_rows_are_null(c1):
    inp = _input(c1)
    g = ra.GRanges(["chr12", "chrUn", "chr12"], [1_000_000, 5, 121_257_000], width=[2000, 2000, 2000])
    cov = ra.calcCoverage(inp[0]["ranges"], g)
    assert cov[1] is None  # not in the reads' seqlevels -> "chrUn not found!" -> NULL
    assert cov[2] is None  # crosses the chromosome end -> subscript error -> NULL


def _runs_ok(rle, dense):
    np.testing.assert_array_equal(rle.decode(), dense)
    assert len(rle.values) == len(rle.lengths)
    assert (rle.lengths > 0).all()
    assert (np.diff(rle.values) != 0).all()  # runs are maximal, as Rle() builds them


def test_calc_coverage_rle(c1):
    """calcCoverage returns Rle objects in the reference (R/coverage.R:171-173)."""
    inp = _input(c1)
    for mask in (c1["genome"], c1["exons"], ra.getRegionalRanges(c1["genome"], "tss", FLANK)):
        dense = ra.calcCoverage(inp[1]["ranges"], mask)
        rle = ra.calcCoverage(inp[1]["ranges"], mask, rle=True)
        assert len(rle) == len(dense)
        for d, e in zip(dense, rle):
            assert (d is None) == (e is None)
            if d is not None:
                _runs_ok(e, d)


def test_rle_edge_rows(c1):
    """Empty (index-0-only) and NULL rows between ordinary ones keep their run offsets."""
    inp = _input(c1)
    g = ra.GRanges(["chr12"] * 5, [0, 1_000_000, -5, 1_000_100, 121_257_000],
                   [0, 1_003_000, 10, 1_000_100, 121_258_000])
    dense = ra.calcCoverage(inp[0]["ranges"], g)
    rle = ra.calcCoverage(inp[0]["ranges"], g, rle=True)
    for d, e in zip(dense, rle):
        assert (d is None) == (e is None)
        if d is not None:
            _runs_ok(e, d)


def test_recoup_profiles_fused_heatmap(c1):
    """recoup() TSS per-base profile + its forced 200-bin heatmap pass (R/recoup.R:659-671),
    computed from one device pass."""
    inp = ra.coverageRef(_input(c1), c1["genome"], "tss", FLANK)
    inp = ra.recoupProfiles(inp, c1["genome"], "tss", FLANK, {"flankBinSize": 0, "regionBinSize": 0})
    for k, s in enumerate(inp):
        np.testing.assert_array_equal(np.asarray(s["profile"]), c1["gold"][f"tss_base_s{k}"].astype(np.float64))
        np.testing.assert_allclose(s["heatmap"], c1["gold"][f"tss_heat_s{k}"], rtol=1e-12, atol=0)


def test_recoup_profiles_genebody(c1):
    inp = ra.coverageRef(_input(c1), c1["genome"], "genebody", FLANK)
    inp = ra.recoupProfiles(inp, c1["genome"], "genebody", FLANK,
                            {"flankBinSize": 50, "regionBinSize": 150, "sumStat": "median"})
    for k, s in enumerate(inp):
        np.testing.assert_allclose(s["profile"], c1["gold"][f"gb_median_s{k}"], rtol=1e-9, atol=1e-12)
        assert "heatmap" not in s
    # the reference's forced heatmap pass of a genebody profile errors (recoup.R:703)
    inp = ra.coverageRef(_input(c1), c1["genome"], "genebody", FLANK)
    with pytest.raises(ra.SemanticError):
        ra.recoupProfiles(inp, c1["genome"], "genebody", FLANK, {"flankBinSize": 0, "regionBinSize": 150})


def test_bam_ingest_to_profile(c1):
    """readBam (R/ranges.R:120-124) -> coverageRef -> profileMatrix on the reference's BAM
    fixtures, against the oracle on the same reads."""
    bams = [os.path.join(os.path.dirname(__file__), "golden", "bam", f)
            for f in ("WT_H4K20me1_50kr.bam", "Set8KO_H4K20me1_50kr.bam")]
    inp = [{"id": f"s{k}", "name": os.path.basename(b), "ranges": ra.readBam(b)} for k, b in enumerate(bams)]
    inp = ra.coverageRef(inp, c1["genome"], "tss", FLANK)
    inp = ra.profileMatrix(inp, FLANK, {"flankBinSize": 0, "regionBinSize": 100})
    win = ra.getRegionalRanges(c1["genome"], "tss", FLANK)
    for s in inp:
        g = s["ranges"]
        ix = o.Index(g.seqcodes, g.start, g.end, g.strand, g.seqlengths)
        mask = o.Mask.from_ranges(win.codes_in(g.seqlevels), win.start, win.end, win.strand)
        ref, rv = o.profile_part(ix, mask, 100)
        np.testing.assert_allclose(s["profile"], ref, rtol=1e-12, atol=0)
        assert s["profile"].sum() > 0


def test_bam_path_input(c1):
    """calcCoverage / coverageRef / coverageRnaRef with a BAM path (R/coverage.R:127-140,
    35-39, 93-96 -> coverageFromBam, :228-295): every mapped alignment overlapping a region,
    strand filter skipped and ignore.strand unused -- the same lists as the readBam reads with
    no filter and strands ignored, whatever strand arguments are passed; the oracle agrees."""
    bam = os.path.join(os.path.dirname(__file__), "golden", "bam", "WT_H4K20me1_50kr.bam")
    reads = ra.readBam(bam)
    win = ra.getRegionalRanges(c1["genome"], "tss", FLANK)
    got = ra.calcCoverage(bam, win, strand="+", ignore_strand=False)
    ref = ra.calcCoverage(reads, win)
    ix = o.Index(reads.seqcodes, reads.start, reads.end, reads.strand, reads.seqlengths)
    mask = o.Mask.from_ranges(win.codes_in(reads.seqlevels), win.start, win.end, win.strand)
    exp = o.coverage(ix, mask, ignore_strand=True)
    assert len(got) == len(ref) == len(exp) == len(win)
    n_valid = 0
    for g, r, e in zip(got, ref, exp):
        assert (g is None) == (r is None) == (e is None)
        if g is not None:
            np.testing.assert_array_equal(g, r)
            np.testing.assert_array_equal(g, e)
            n_valid += 1
    assert n_valid > 0
    # coverageRef / coverageRnaRef on samples that carry only the file
    inp = ra.coverageRef([{"id": "s0", "name": "WT", "file": bam}], c1["genome"], "tss", FLANK,
                         strandedParams={"strand": "-", "ignoreStrand": False})
    inp = ra.profileMatrix(inp, FLANK, {"flankBinSize": 0, "regionBinSize": 100})
    ref_p, _ = o.profile_part(ix, mask, 100)
    np.testing.assert_allclose(inp[0]["profile"], ref_p, rtol=1e-12, atol=0)
    rna_f = ra.coverageRnaRef([{"id": "s0", "name": "WT", "file": bam}], c1["exons"], c1["genome"], FLANK)
    rna_r = ra.coverageRnaRef([{"id": "s0", "name": "WT", "ranges": reads}], c1["exons"], c1["genome"], FLANK)
    for g, r in zip(rna_f[0]["coverage"].to_list(), rna_r[0]["coverage"].to_list()):
        assert (g is None) == (r is None)
        if g is not None:
            np.testing.assert_array_equal(g, r)
    with pytest.raises(ValueError):
        ra.calcCoverage(os.path.join(os.path.dirname(__file__), "golden", "nope.bam"), win)
