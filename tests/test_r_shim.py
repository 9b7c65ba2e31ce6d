"""The R side of the drop-in boundary (r/src/recoup_amd_shim.c, r/R/rcp.R), without R.

* The .Call shim compiles against include/recoup_amd.h (tests/rstub declares the R C API it
  uses); every routine the R wrappers .Call is registered, with the arity of its C signature;
  the shim calls only header symbols.
* The shim is EXECUTED through tests/rmini (a small emulation of the R C API): the host-only
  routines here (BAM ingest, the preprocessing RNG, the no-device error), the GPU ones in
  tests/test_gpu_rshim.py.  With allocation failures injected at every R allocation the shim
  makes, no library handle is ever left outside a finalizer-backed external pointer.
* Every calcCoverage call site of the reference (R/coverage.R) passes an input type rcp.R's
  calcCoverage accepts, and rcp.R replaces coverageRnaRef / coverageAreaRef / coverageBaseRef.
* tests/r_mirror.py (the Python transliteration of rcp.R the GPU tests drive) mirrors functions
  that exist in rcp.R, and its row tables equal the Python API's (tested on the GPU)."""
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHIM = os.path.join(ROOT, "r", "src", "recoup_amd_shim.c")
RSRC = os.path.join(ROOT, "r", "R", "rcp.R")
REF_COVERAGE = "/root/reference/R/coverage.R"
BAM = os.path.join(ROOT, "tests", "golden", "bam", "WT_H4K20me1_50kr.bam")


def test_shim_compiles_against_the_header():
    r = subprocess.run(["gcc", "-std=c99", "-Wall", "-Wextra", "-Werror", "-Wno-unused-parameter",
                        "-Wno-cast-function-type", "-fsyntax-only", "-I", os.path.join(ROOT, "tests", "rstub"),
                        "-I", os.path.join(ROOT, "include"), SHIM], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def _registrations():
    shim = open(SHIM).read()
    return dict((n, int(k)) for n, k in re.findall(r'\{"(rcp_R_\w+)", \(DL_FUNC\)&\w+, (\d+)\}', shim))


def test_registered_routines_cover_the_r_wrappers():
    shim = open(SHIM).read()
    reg = _registrations()
    for name, nargs in reg.items():  # registration arity = C signature arity
        sig = re.search(r"SEXP %s\(([^)]*)\)" % name, shim).group(1)
        assert sig.count("SEXP") == nargs, name
    called = set(re.findall(r'"(rcp_R_\w+)"', open(RSRC).read()))
    assert called and called <= set(reg), called - set(reg)


def test_shim_calls_only_header_symbols():
    from tests.test_abi import header_symbols
    shim = open(SHIM).read()
    used = set(re.findall(r"\b(rcp_[a-z_]+)\(", shim)) - set(re.findall(r"(rcp_R_\w+)", shim))
    used -= {"rcp_rows_desc", "rcp_bins_desc"}
    assert used <= set(header_symbols()), used - set(header_symbols())


# ---------------------------------------------------------------- handles vs R allocations
HANDLE_CALLS = r"rcp_readset_create\(|rcp_readset_create_multi\(|rcp_coverage_rle\(|rcp_bam_read\(|rcp_rng_create\("
R_ALLOCS = r"\b(allocVector|allocMatrix|R_alloc|mkChar|R_MakeExternalPtr|new_guard|wrap_\w+)\("


def _bodies(src):
    """name -> body of every SEXP-returning function of the shim."""
    out = {}
    for m in re.finditer(r"\nSEXP (rcp_R_\w+)\([^)]*\)\s*\{", src):
        i, depth = m.end(), 1
        while depth:
            depth += {"{": 1, "}": -1}.get(src[i], 0)
            i += 1
        out[m.group(1)] = src[m.end():i]
    return out


def test_no_raw_handle_is_live_across_an_r_allocation():
    """Statically: after each library call that hands out a handle, the handle is stored in an
    external pointer with a finalizer (R_SetExternalPtrAddr) before the next R allocation or
    Rf_error (check)."""
    bodies = _bodies(open(SHIM).read())
    seen = 0
    for name, body in bodies.items():
        for m in re.finditer(HANDLE_CALLS, body):
            seen += 1
            rest = body[m.end():]
            guard = rest.find("R_SetExternalPtrAddr")
            assert guard >= 0, f"{name}: handle never stored in an external pointer"
            nxt = re.search(R_ALLOCS + r"|\bcheck\(", rest)
            assert nxt is None or guard < nxt.start(), f"{name}: R allocation or error before the handle is guarded"
            # the guard itself was made before the call (the call site cannot allocate after it)
            assert "new_guard(" in body[:m.start()], f"{name}: guard not made before the library call"
    assert seen >= 5


# ---------------------------------------------------------------- executing the shim (host)
@pytest.fixture(scope="module")
def sh():
    from tests.rmini import rmini
    rmini.build()
    return rmini.shim()


def test_every_r_wrapper_routine_is_callable(sh):
    for name, k in _registrations().items():
        assert sh.routine_arity(name) == k, name


def test_read_bam_through_the_shim(sh):
    from recoup_amd import api
    r = sh.call("rcp_R_read_bam", BAM, np.int32(0), 0.75, np.int32(4))
    g = api.readBam(BAM, "keep")
    assert r["seqnames"] == list(g.seqlevels)
    np.testing.assert_array_equal(r["seqlengths"], g.seqlengths.astype(np.float64))
    np.testing.assert_array_equal(r["chrom"], g.seqcodes)
    np.testing.assert_array_equal(r["start"], g.start)
    np.testing.assert_array_equal(r["end"], g.end)
    np.testing.assert_array_equal(r["strand"], g.strand)
    assert sh.live_handles() == 0  # the BAM handle was released before returning


def test_sample_sorted_through_the_shim(sh):
    from tests import rrng
    res = sh.call("rcp_R_sample_sorted", np.int32(42), np.int32(0), np.array([1000.0, 5000.0]), 100.0)
    g = rrng.RRng(42, "Rejection")
    for got, n in zip(res, (1000, 5000)):
        np.testing.assert_array_equal(got, np.sort(g.sample_int(n, 100)).astype(np.float64))


@pytest.mark.parametrize("routine", ["rcp_R_read_bam", "rcp_R_sample_sorted"])
def test_allocation_failures_never_leak_a_handle(sh, routine):
    """R raises an error when it cannot allocate; inject that failure at every allocation the
    routine makes, one run each: the library handle is then always held by an external pointer
    whose finalizer releases it (the garbage collector's job in R)."""
    from tests.rmini import rmini
    args = {"rcp_R_read_bam": (BAM, np.int32(0), 0.75, np.int32(2)),
            "rcp_R_sample_sorted": (np.int32(42), np.int32(0), np.array([1000.0, 5000.0]), 100.0)}[routine]
    failures = 0
    for k in range(200):
        sh.fail_alloc_after(k)
        try:
            sh.call(routine, *args)
            sh.fail_alloc_after(-1)
            break
        except rmini.RError as e:
            assert "injected" in str(e), e
            failures += 1
            assert sh.unguarded_handles() == 0, f"allocation {k}: a library handle is held by nothing"
            sh.run_finalizers()
            assert sh.live_handles() == 0, f"allocation {k}: a finalizer left its handle"
    else:
        pytest.fail("the routine never completed")
    assert failures >= 3


def test_no_device_error_unwinds_cleanly(sh):
    import torch
    from tests.rmini import rmini
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    with pytest.raises(rmini.RError, match="no HIP device"):
        sh.call("rcp_R_readset", np.zeros(3, np.int32), np.array([1, 5, 9], np.int32),
                np.array([10, 20, 30], np.int32), np.zeros(3, np.int32), np.array([100.0]), np.int32(-1),
                np.int32(0))
    assert sh.unguarded_handles() == 0


# ---------------------------------------------------------------- the reference's call sites
# calcCoverage calls of R/coverage.R (line: first argument, the input types it can carry).
# theRanges is splitBySeqname's per-chromosome list (:54, :95) or, in coverageRnaRef, a
# sample's BAM path (:97).
CALL_SITES = {
    33: ("input[[n]]$ranges", {"GRanges"}),
    37: ("input[[n]]$file", {"BAM path"}),
    55: ("theRanges", {"split list"}),
    60: ("input[[n]]$file", {"BAM path"}),
    101: ("theRanges", {"split list", "BAM path"}),
    106: ("theRanges", {"split list", "BAM path"}),
    111: ("theRanges", {"split list", "BAM path"}),
}


def _r_function(src, name):
    """The text of an R function of rcp.R: its definition up to its closing brace at column 0
    (or, for a one-expression body, up to the next top-level line)."""
    m = re.search(r"^%s <- function\(" % re.escape(name), src, re.M)
    assert m, f"{name} is not defined in rcp.R"
    lines = src[m.start():].split("\n")
    out = [lines[0]]
    for ln in lines[1:]:
        if ln and not ln[0].isspace():
            if ln.startswith("}"):
                out.append(ln)
            break
        out.append(ln)
    return "\n".join(out)


def test_reference_call_sites_are_the_ones_listed():
    if not os.path.exists(REF_COVERAGE):
        pytest.skip("the reference is not present (GPU box)")
    sites = {}
    for i, line in enumerate(open(REF_COVERAGE), 1):
        code = line.split("#", 1)[0]
        m = re.search(r"calcCoverage\(([^,]+),", code)
        if m and "<- function" not in code:
            sites[i] = m.group(1).strip()
    assert sites == {k: v[0] for k, v in CALL_SITES.items()}


def test_calc_coverage_accepts_every_reference_input():
    src = open(RSRC).read()
    cc = _r_function(src, "calcCoverage")
    args = _r_function(src, ".rcpReadArgs")
    # the reference's own input check is kept, so a list passes it (R/coverage.R:127-130)
    assert '!is(input, "GRanges") && !is.list(input) && is.character(input)' in cc
    handles = {
        "GRanges": 'is(input, "GRanges")' in args and "input <- list(input)" in args,
        "split list": "Reduce(merge, lapply(unname(input), seqinfo))" in args
                      and "input[!vapply(input, is.null, TRUE)]" in args,
        "BAM path": "is.character(input)" in cc and ".rcpReadBam(input)" in cc,
    }
    for line, (arg, types) in CALL_SITES.items():
        for t in types:
            assert handles[t], f"R/coverage.R:{line} passes {arg} as a {t}, which rcp.R's calcCoverage rejects"
    assert ".rcpReadSet(input, strand" in cc  # GRanges / list: the strand filter is the readset's


def test_rcp_replaces_the_coverage_callers():
    """coverageRnaRef's three calcCoverage passes + c() merge are one pass per sample over one
    readset; coverageAreaRef does not split the reads in R."""
    src = open(RSRC).read()
    rna = _r_function(src, "coverageRnaRef")
    assert rna.count(".rcpSampleReadSet(") == 1 and rna.count(".rcpCoverage(") == 1
    assert "calcCoverage(" not in rna
    assert ".rcpRnaRows(" in rna and "flank[1] == 0" in rna
    for f in ("coverageAreaRef", "coverageBaseRef"):
        assert ".rcpCoverageRef(" in _r_function(src, f)
    ref = _r_function(src, ".rcpCoverageRef")
    assert "splitBySeqname" not in ref and ref.count(".rcpCoverage(") == 1


def test_mirror_names_exist_in_rcp_r():
    from tests import r_mirror
    src = open(RSRC).read()
    for name in r_mirror.MIRRORED:
        assert re.search(r"^%s <- function\(" % re.escape(name), src, re.M), name


def test_mirror_rna_rows_equal_the_api_rows():
    """.rcpRnaRows (through its mirror) builds the row table the Python API's coverageRnaRef
    builds -- the one the GPU parity tests cover."""
    from recoup_amd import api
    from recoup_amd.granges import GRanges, GRangesList, getFlankingRanges
    from tests import r_mirror
    from tests.golden import c1_cases
    d = c1_cases.load_inputs()
    G, E = c1_cases.genome(d), c1_cases.exons(d)
    genes = GRanges(G["chrom"], G["start"], G["end"], G["strand"], names=G["names"])
    flat = GRanges(E["chrom"], E["start"], E["end"], E["strand"])
    exons = GRangesList(flat, E["seg_off"], names=E["names"])
    levels = ["chr12", "chrX"]
    for flank in ((2000, 2000), (0, 500), (1000, 0)):
        left = getFlankingRanges(genes, 1 if flank[0] == 0 else flank[0], "upstream")
        right = getFlankingRanges(genes, 1 if flank[0] == 0 else flank[1], "downstream")
        rows = r_mirror.rcp_rna_rows(left, exons, right, levels, True)
        ref = api._rna_rows(exons, genes, flank, levels, True)
        np.testing.assert_array_equal(rows["segOff"], ref.seg_off)
        chrom = np.where(rows["chrom"] == np.iinfo(np.int32).min, -1, rows["chrom"])
        np.testing.assert_array_equal(chrom, ref.chrom)
        np.testing.assert_array_equal(rows["start"], ref.start)
        np.testing.assert_array_equal(rows["end"], ref.end)
        np.testing.assert_array_equal(rows["strand"], ref.strand)
        np.testing.assert_array_equal(rows["group"], ref.seg_group)
        np.testing.assert_array_equal(rows["isList"], ref.group_is_list.astype(bool))


def test_mirror_read_args_of_a_split_list():
    """A splitBySeqname list and its GRanges give the same reads (grouped by chromosome), the
    same merged seqinfo and width runs."""
    from recoup_amd.granges import GRanges
    from tests import r_mirror
    rng = np.random.default_rng(3)
    n = 5000
    chrom = rng.choice(["chr1", "chr2", "chr3"], n)
    start = rng.integers(1, 100000, n)
    g = GRanges(chrom, start, start + 99, rng.integers(0, 3, n), seqlevels=["chr1", "chr2", "chr3", "chrM"],
                seqlengths={"chr1": 200000, "chr3": 150000})
    sp = r_mirror.split_by_seqname(g)
    assert list(sp) == ["chr1", "chr2", "chr3"]
    lv, args = r_mirror.rcp_read_args(sp)
    lv1, args1 = r_mirror.rcp_read_args(g)
    assert lv == lv1 == ["chr1", "chr2", "chr3", "chrM"]
    np.testing.assert_array_equal(args[4], args1[4])  # seqlengths (NA for chr2, chrM)
    assert isinstance(args[2], list) and list(args[2][0]) == [100]  # one width run
    vals, lens = args[0]
    np.testing.assert_array_equal(vals, [0, 1, 2])  # one run per chromosome
    order = np.argsort(g.seqcodes, kind="stable")
    np.testing.assert_array_equal(args[1], g.start[order])
    np.testing.assert_array_equal(args[3], g.strand[order])


# ---------------------------------------------------------------- profile shapes (dimnames)
def test_profile_dimnames_rules():
    """The oracle's restatement of the dimnames R leaves on profileMatrix's matrix."""
    from oracle import oracle as o
    names = ["g1", "g2", "g3"]
    assert o.bin_colnames(3, "mean") == ["1.mean", "2.mean", "3.mean"]
    # equal lengths: rbind of the named list
    assert o.profile_dimnames(names, (2000, 2000), dict(regionBinSize=0), True) == (names, None)
    assert o.profile_dimnames(names, (2000, 2000), dict(regionBinSize=2, sumStat="median"), True) == \
        (names, ["1.median", "2.median"])
    assert o.profile_dimnames(None, (2000, 2000), dict(regionBinSize=0), True) is None
    assert o.profile_dimnames(None, (2000, 2000), dict(regionBinSize=1), True) == (None, ["1.mean"])
    # unequal: cbind(left, center, right) + rownames<-; flank bins round(2 * fbs * f / sum(f))
    dn = o.profile_dimnames(names, (3000, 1000), dict(flankBinSize=2, regionBinSize=2), False)
    assert dn == (names, ["1.mean", "2.mean", "3.mean", "1.mean", "2.mean", "1.mean"])
    dn = o.profile_dimnames(names, (2, 0), dict(flankBinSize=0, regionBinSize=1), False)
    assert dn == (names, ["", "", "1.mean"])


def test_r_cbind_model():
    from tests import r_mirror as rm
    from tests.rmini.rmini import RArray
    a = RArray(np.zeros((2, 2)))
    b = RArray(np.ones((2, 1)), (None, ["1.mean"]))
    m = rm.r_cbind(None, a, b)
    assert m.shape == (2, 3) and m.dimnames == (None, ["", "", "1.mean"])
    assert rm.r_set_rownames(m, ["x", "y"]).dimnames == (["x", "y"], ["", "", "1.mean"])
    assert rm.r_cbind(a, a).dimnames is None
    assert rm.r_set_rownames(a, None).dimnames is None


def test_rcp_replaces_profile_matrix():
    """profileMatrix keeps the reference's signature (R/profile.R:1) and makes one library call
    per sample in the unequal-length branch; the binning functions name rows as the reference's
    rbind does: by names(cvrg) when mapping over cvrg itself, not over the slices."""
    src = open(RSRC).read()
    pm = _r_function(src, "profileMatrix")
    assert pm.startswith("profileMatrix <- function(input, flank, binParams, rc = NULL) {")
    assert "for (n in names(input))" in pm and "if (!any(hasProfile))" in pm
    assert pm.count(".rcpProfileRle(") == 1 and "names(cvrg))" in pm
    assert "binCoverageMatrix(cvrg, binSize = binParams$regionBinSize" in pm
    bcm = _r_function(src, "binCoverageMatrix")
    assert "if (is.null(flank)) names(cvrg) else NULL" in bcm
    base = _r_function(src, "baseCoverageMatrix")
    assert "rowNames = names(cvrg)" in base
    assert "profileMatrixFused" not in src
    shim = open(SHIM).read()
    # every profile routine sets the dimnames of the matrix it returns
    for name, body in _bodies(shim).items():
        if "allocMatrix" in body:
            assert "set_dimnames(" in body, name
