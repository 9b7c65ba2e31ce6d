"""Line-by-line Python transliterations of the R wrappers in r/R/rcp.R (test infrastructure).

R is not installed here or on the GPU box, so the R functions themselves cannot run.  These
mirrors build exactly the ``.Call`` arguments the R code builds -- same vectors, same types
(integer / double / logical), same order -- from the Python GRanges stand-ins, and drive the
real shim through tests/rmini (an emulation of the R C API).  Each function names the R
function it mirrors; a change to rcp.R must be reflected here (tests/test_r_shim.py checks
that every mirrored R function still exists).
"""
import numpy as np

from recoup_amd.granges import GRanges, GRangesList, getFlankingRanges, getRegionalRanges

MIRRORED = [".rcpDevices", ".rcpReadArgs", ".rcpReadSet", ".rcpFree", ".rcpSampleReadSet", ".rcpRows", ".rcpRowArgs",
            ".rcpCoverage", "calcCoverage", ".rcpCoverageRef", ".rcpRnaRows", "coverageRnaRef", ".rcpRleArrays",
            ".rcpProfileRle", ".rcpStrandOfListError", "binCoverageMatrix", "baseCoverageMatrix", ".rcpParts", "profileMatrix",
            "profileMatrixFromReads"]


class NamedList(list):
    """An R list with names (None = no names attribute), e.g. calcCoverage's list of Rle.
    ``rcp_runs``: its attr(, "rcpRuns") (the device handle of the runs and their addresses), or
    None -- R keeps the attribute when an element is replaced, not when the list is rebuilt."""

    def __init__(self, items, names=None):
        super().__init__(items)
        self.names = None if names is None else [str(x) for x in names]
        self.rcp_runs = None


class Rle(tuple):
    """An S4Vectors::Rle: (runValue, runLength), with ``robj`` the R object (an rmini S4 object
    with slots values / lengths) the shim sees -- one per Rle, as R's object identity."""

    def __new__(cls, values, lengths, sh=None):
        obj = super().__new__(cls, (values, lengths))
        obj.robj = None if sh is None else sh.s4(values=np.asarray(values, np.int32) if np.asarray(values).dtype.kind
                                                 in "iu" else np.asarray(values, np.float64),
                                                 lengths=np.asarray(lengths, np.int32))
        return obj


# options(recoup.deviceRuns): calcCoverage's runs stay on the device beside the list (default TRUE)
DEVICE_RUNS = True
KEPT = []    # the handles the lists hold (R frees them when it collects the lists)
PATHS = []   # .rcpProfileRle's choice per call: "device" (rcp_R_profile_cov) or "upload"


def kept_alive(sh):
    """Coverage handles still holding device runs (what R's garbage collector would release)."""
    return sum(bool(sh.call("rcp_R_cov_alive", h)[0]) for h in KEPT)


def rle_addresses(sh, cvrg):
    """.Call("rcp_R_rle_addresses", cvrg)."""
    return sh.call("rcp_R_rle_addresses", [getattr(x, "robj", None) for x in cvrg])


def _rchar(names):
    """An R character vector for the shim, or NULL."""
    from tests.rmini.rmini import RChar
    return None if names is None else RChar(names)


def rle(x):
    """S4Vectors::Rle(x): (runValue, runLength)."""
    x = np.asarray(x)
    if x.size == 0:
        return x[:0], np.zeros(0, np.int64)
    brk = np.nonzero(x[1:] != x[:-1])[0] + 1
    starts = np.concatenate([[0], brk])
    return x[starts], np.diff(np.concatenate([starts, [x.size]]))


def split_by_seqname(gr):
    """splitBySeqname (R/util.R:1-13): level -> reads on it (empty levels dropped); each
    element keeps the whole seqinfo, as GRanges subsetting does."""
    out = {}
    for c, lv in enumerate(gr.seqlevels):
        sel = gr.seqcodes == c
        if sel.any():
            out[lv] = gr[sel]
    return out


def merge_seqinfo(grs):
    """Reduce(merge, lapply(input, seqinfo)): union of seqlevels in first-seen order; a length
    known in one element and NA in another is known."""
    levels, sl = [], {}
    for g in grs:
        for lv, n in zip(g.seqlevels, g.seqlengths):
            if lv not in sl:
                levels.append(lv)
                sl[lv] = -1
            if n >= 0:
                if sl[lv] >= 0 and sl[lv] != n:
                    raise ValueError(f"incompatible seqlengths for {lv}")
                sl[lv] = int(n)
    return levels, sl


def rcp_read_args(inp, levels=None):
    """.rcpReadArgs(input, levels): (levels, list(chrom, start, ends, strand, seqlengths))."""
    if isinstance(inp, GRanges):
        inp = [inp]
    elif isinstance(inp, dict):
        inp = list(inp.values())
    inp = [g for g in inp if g is not None]
    lv_all, sl = merge_seqinfo(inp)
    lv = lv_all if levels is None else list(levels)
    if len(lv) == 0:
        return ["."], [np.zeros(0, np.int32)] * 4 + [np.array([np.nan])]
    code = {c: i for i, c in enumerate(lv)}
    rv, rl = [], []
    for g in inp:
        names = np.array(g.seqlevels, dtype=object)[g.seqcodes] if len(g) else np.array([], dtype=object)
        v, l = rle(np.array([code[c] for c in names], dtype=np.int32))  # match(...) - 1L
        rv.append(v)
        rl.append(l)
    chrom = [np.concatenate(rv).astype(np.int32) if rv else np.zeros(0, np.int32),
             np.concatenate(rl).astype(np.float64) if rl else np.zeros(0)]
    width = np.concatenate([g.width for g in inp]).astype(np.int32) if inp else np.zeros(0, np.int32)
    wv, wl = rle(width)
    n = width.size
    if len(chrom[0]) > n // 4:  # about a run per read (unsorted): one code per read
        chrom = np.repeat(chrom[0], chrom[1].astype(np.int64)).astype(np.int32)
    elif chrom[1].sum() == 0:
        chrom = np.zeros(0, np.int32)
    if n > 0 and wv.size <= n // 4:
        ends = [wv.astype(np.int32), wl.astype(np.float64)]
    else:
        ends = np.concatenate([g.end for g in inp]).astype(np.int32) if inp else np.zeros(0, np.int32)
    st = np.concatenate([g.start for g in inp]).astype(np.int32) if inp else np.zeros(0, np.int32)
    sd = np.concatenate([g.strand for g in inp]).astype(np.int32) if inp else np.zeros(0, np.int32)
    seqlen = np.array([sl[c] if sl.get(c, -1) >= 0 else np.nan for c in lv], dtype=np.float64)
    return lv, [chrom, st, ends, sd, seqlen]


# options(recoup.devices): set by the tests (getOption's value)
DEVICES = (0,)


def rcp_devices():
    """.rcpDevices()."""
    return tuple(DEVICES)


class ReadSet:
    """The R "rcpReadSet": list(ptr, levels, strand[, rows])."""

    def __init__(self, ptr, levels, strand, rows=None):
        self.ptr, self.levels, self.strand, self.rows = ptr, levels, strand, rows


STRAND = {"+": 0, "-": 1, "*": 2}


def rcp_read_set(sh, inp, strand=None, devices=None, levels=None, rows_of=None):
    """.rcpReadSet(input, strand, devices, levels, rowsOf)."""
    devices = rcp_devices() if devices is None else tuple(devices)
    lv, args = rcp_read_args(inp, levels)
    sf = -1 if strand is None else STRAND[strand]
    if len(devices) > 1 and rows_of is not None:
        rows = rows_of(lv)
        ptr = sh.call("rcp_R_shards", *args, np.int32(sf), *rcp_row_args(rows), np.asarray(devices, np.int32))
        return ReadSet(ptr, lv, strand, rows)
    if len(devices) > 1:
        ptr = sh.call("rcp_R_readsets", *args, np.int32(sf), np.asarray(devices, np.int32), raw=False)
    else:
        ptr = sh.call("rcp_R_readset", *args, np.int32(sf), np.int32(devices[0]))
    return ReadSet(ptr, lv, strand)


def rcp_free(sh, rs):
    """.rcpFree(rs)."""
    if rs.rows is not None:
        sh.call("rcp_R_shards_free", rs.ptr)
        return
    for p in (rs.ptr if isinstance(rs.ptr, list) else [rs.ptr]):
        sh.call("rcp_R_free", p)


def rcp_rows(mask, levels, ignore_strand=True):
    """.rcpRows(mask, levels, ignore.strand)."""
    if isinstance(mask, GRangesList):
        flat, n = mask.flat, np.diff(mask.offsets)
    else:
        flat, n = mask, np.ones(len(mask), np.int64)
    seg_off = np.concatenate([[0.0], np.cumsum(n.astype(np.float64))])
    codes = flat.codes_in(levels)  # match(..., levels) - 1L; NA -> R's NA_integer_
    chrom = np.where(codes < 0, np.iinfo(np.int32).min, codes).astype(np.int32)
    return dict(segOff=seg_off, chrom=chrom, start=flat.start.astype(np.int32), end=flat.end.astype(np.int32),
                strand=flat.strand.astype(np.int32), group=np.zeros(len(flat), np.int32),
                isList=np.array([isinstance(mask, GRangesList), False, False, False]),
                ignoreStrand=np.array([bool(ignore_strand)]))


def rcp_row_args(rows):
    """.rcpRowArgs(rows)."""
    return [rows[k] for k in ("segOff", "chrom", "start", "end", "strand", "group", "isList", "ignoreStrand")]


def rcp_coverage(sh, rs, rows, names=None):
    """.rcpCoverage(rs, rows, names): named list of (values, lengths) runs or None."""
    if rs.rows is not None:
        res = sh.call("rcp_R_shards_coverage", rs.ptr)
    else:
        ptr = rs.ptr[0] if isinstance(rs.ptr, list) else rs.ptr
        res = sh.call("rcp_R_coverage", ptr, *rcp_row_args(rows))
    cov = []
    for r in range(len(res["valid"])):
        if not res["valid"][r]:
            cov.append(None)
            continue
        a, b = int(res["runOff"][r]), int(res["runOff"][r + 1])
        cov.append(Rle(res["values"][a:b], res["lengths"][a:b], sh))
    cov = NamedList(cov, names)
    if DEVICE_RUNS:
        cov.rcp_runs = dict(handle=res["handle"], addr=rle_addresses(sh, cov))
        KEPT.append(res["handle"])
    else:
        sh.call("rcp_R_cov_free", res["handle"])
    return cov


class RStop(Exception):
    """An R stop() raised by the R code mirrored here."""


def rcp_strand_of_list_error():
    """.rcpStrandOfListError()."""
    raise RStop("unable to find an inherited method for function 'strand' for signature '\"list\"'")


def _rows_identical(a, b):
    """identical() of two .rcpRows lists."""
    return a.keys() == b.keys() and all(np.array_equal(np.asarray(a[k]), np.asarray(b[k])) for k in a)


def calc_coverage(sh, inp, mask, strand=None, ignore_strand=True):
    """calcCoverage(input, mask, strand, ignore.strand) for a GRanges, a split list or a readset
    the caller prepared (.rcpReadSet)."""
    own = not isinstance(inp, ReadSet)
    if not own:
        if strand != inp.strand:
            raise RStop("the readset was prepared with another strand filter")
        if inp.rows is not None and not _rows_identical(inp.rows, rcp_rows(mask, inp.levels, ignore_strand)):
            raise RStop("the readset was split over the devices for another mask")
        rs = inp
    else:
        if strand is not None and not isinstance(inp, GRanges):
            rcp_strand_of_list_error()
        rs = rcp_read_set(sh, inp, strand, rows_of=lambda lv: rcp_rows(mask, lv, ignore_strand))
    try:
        return rcp_coverage(sh, rs, rs.rows if rs.rows is not None else rcp_rows(mask, rs.levels, ignore_strand),
                            mask.names)
    finally:
        if own:
            rcp_free(sh, rs)


def coverage_ref(sh, input, genomeRanges, region, flank, strandedParams, split=False):
    """.rcpCoverageRef (coverageBaseRef / coverageAreaRef: split = TRUE)."""
    main = getRegionalRanges(genomeRanges, region, flank)
    for x in input:
        if split and x.get("ranges") is not None and strandedParams.get("strand") is not None:
            rcp_strand_of_list_error()
        ign = strandedParams.get("ignoreStrand", True)  # .rcpSampleReadSet
        rs = rcp_read_set(sh, x["ranges"], strandedParams.get("strand"), rows_of=lambda lv: rcp_rows(main, lv, ign))
        rows = rs.rows if rs.rows is not None else rcp_rows(main, rs.levels, ign)
        x["coverage"] = rcp_coverage(sh, rs, rows, main.names)
        rcp_free(sh, rs)
    return input


def rcp_rna_rows(left, exons, right, levels, ignore_strand=True):
    """.rcpRnaRows(left, exons, right, levels, ignore.strand)."""
    G = len(exons)
    if len(left) != G or len(right) != G:
        raise ValueError("helperRanges and genomeRanges differ in length")
    nex = np.diff(exons.offsets)
    flat = exons.flat
    seg_off = np.concatenate([[0.0], np.cumsum((nex + 2).astype(np.float64))])
    n = int(seg_off[G])
    first = seg_off[:-1].astype(np.int64)  # R's first - 1 (0-based here)
    last = seg_off[1:].astype(np.int64) - 1
    is_ex = np.ones(n, bool)
    is_ex[np.concatenate([first, last])] = False

    def code(g):
        c = g.codes_in(levels)
        return np.where(c < 0, np.iinfo(np.int32).min, c)

    chrom, st, en, sd = (np.zeros(n, np.int32) for _ in range(4))
    grp = np.ones(n, np.int32)
    chrom[first], st[first], en[first], sd[first], grp[first] = code(left), left.start, left.end, left.strand, 0
    chrom[last], st[last], en[last], sd[last], grp[last] = code(right), right.start, right.end, right.strand, 2
    chrom[is_ex], st[is_ex], en[is_ex], sd[is_ex] = code(flat), flat.start, flat.end, flat.strand
    return dict(segOff=seg_off, chrom=chrom, start=st, end=en, strand=sd, group=grp,
                isList=np.array([False, True, False, False]), ignoreStrand=np.array([bool(ignore_strand)]))


def coverage_rna_ref(sh, input, genomeRanges, helperRanges, flank, strandedParams=None):
    """coverageRnaRef(input, genomeRanges, helperRanges, flank, strandedParams)."""
    sp = strandedParams or {"strand": None, "ignoreStrand": True}
    left = getFlankingRanges(helperRanges, 1 if flank[0] == 0 else flank[0], "upstream")
    right = getFlankingRanges(helperRanges, 1 if flank[0] == 0 else flank[1], "downstream")
    for x in input:
        if x.get("ranges") is not None and sp.get("strand") is not None:
            rcp_strand_of_list_error()
        ign = sp.get("ignoreStrand", True)

        def rows_of(lv):
            return rcp_rna_rows(left, genomeRanges, right, lv, ign)
        rs = rcp_read_set(sh, x["ranges"], sp.get("strand"), rows_of=rows_of)
        rows = rs.rows if rs.rows is not None else rows_of(rs.levels)
        x["coverage"] = rcp_coverage(sh, rs, rows, genomeRanges.names)
        rcp_free(sh, rs)
    return input


def rcp_rle_arrays(cvrg):
    """.rcpRleArrays(cvrg): runOff, values, lengths, isNull."""
    is_null = np.array([x is None for x in cvrg])
    nr = np.array([0 if x is None else len(x[0]) for x in cvrg], np.float64)
    vals = [x[0] for x in cvrg if x is not None]
    values = np.concatenate(vals) if vals else np.zeros(0, np.int32)
    values = values.astype(np.int32) if values.dtype.kind in "iu" else values.astype(np.float64)
    lengths = np.concatenate([x[1] for x in cvrg if x is not None]).astype(np.int32) if vals else np.zeros(0, np.int32)
    return dict(runOff=np.concatenate([[0.0], np.cumsum(nr)]), values=values, lengths=lengths, isNull=is_null)


STAT = {"mean": 0, "median": 1}
INTERP = {"auto": 0, "spline": 1, "linear": 2, "neighborhood": 3}


def rcp_profile_rle(sh, cvrg, where, flank, n_bins, per_base, stat="mean", interpolation="auto", rng_kind=0,
                    row_names=None):
    """.rcpProfileRle(cvrg, where, flank, nBins, perBase, stat, interpolation, rowNames): the
    matrix (an rmini RArray carrying the dimnames the shim set) -- from the runs still on the
    device when the list is the one calcCoverage returned (its rcpRuns handle alive, its Rle
    vectors at the recorded addresses), else from its Rle vectors uploaded."""
    bin_args = [np.asarray(where, np.int32), np.asarray((0, 0) if flank is None else flank, np.int32),
                np.asarray(n_bins, np.int32), np.asarray(per_base, np.int32), np.int32(STAT[stat]),
                np.int32(INTERP[interpolation]), np.int32(rng_kind), 1.0]
    h = getattr(cvrg, "rcp_runs", None)
    if h is not None and sh.call("rcp_R_cov_alive", h["handle"])[0] and \
            np.array_equal(rle_addresses(sh, cvrg), h["addr"]):
        PATHS.append("device")
        return sh.call("rcp_R_profile_cov", h["handle"], *bin_args, _rchar(row_names))["profile"]
    PATHS.append("upload")
    a = rcp_rle_arrays(cvrg)
    res = sh.call("rcp_R_profile_rle", a["runOff"], a["values"], a["lengths"], a["isNull"], *bin_args,
                  np.asarray(rcp_devices(), np.int32), _rchar(row_names))
    return res["profile"]


def _names(cvrg):
    return getattr(cvrg, "names", None)


WHERE = {"center": 1, "upstream": 2, "downstream": 3}


def bin_coverage_matrix(sh, cvrg, binSize=1000, stat="mean", interpolation="auto", flank=None, where="center"):
    """binCoverageMatrix(cvrg, binSize, stat, interpolation, flank, where)."""
    w = 0 if flank is None else WHERE[where]
    return rcp_profile_rle(sh, cvrg, [w], flank, [binSize], [0], stat, interpolation,
                           row_names=_names(cvrg) if flank is None else None)


def base_coverage_matrix(sh, cvrg, flank=None, where="upstream"):
    """baseCoverageMatrix(cvrg, flank, where)."""
    if flank is None:
        ok = [i for i, x in enumerate(cvrg) if x is not None and int(np.sum(x[1])) > 0]
        size = int(np.sum(cvrg[ok[0]][1])) if ok else 0
        return rcp_profile_rle(sh, cvrg, [0], None, [0], [size], row_names=_names(cvrg))
    w = {"upstream": 1, "downstream": 2}[where]
    return rcp_profile_rle(sh, cvrg, [w + 1], flank, [0], [flank[w - 1]])


def rcp_parts(equal, len1, flank, binParams):
    """.rcpParts(equal, len1, flank, binParams)."""
    if equal:
        rbs = binParams["regionBinSize"]
        return dict(where=[0], nBins=[rbs], perBase=[len1 if rbs == 0 else 0])
    where, nb, pb = [1], [binParams["regionBinSize"]], [0]
    r = np.asarray(flank, np.float64) / sum(flank)
    for k in (0, 1):
        if flank[k] == 0:
            continue
        fb = int(np.round(2 * binParams["flankBinSize"] * r[k])) if binParams["flankBinSize"] != 0 else 0
        if binParams["flankBinSize"] != 0 and fb == 0:
            raise ValueError("invalid 'size' argument")
        if k == 0:
            where, nb, pb = [2] + where, [fb] + nb, [0 if fb else flank[0]] + pb
        else:
            where, nb, pb = where + [3], nb + [fb], pb + [0 if fb else flank[1]]
    return dict(where=where, nBins=nb, perBase=pb)


def _lengths(cvrg):
    return np.array([0 if x is None else int(np.sum(x[1])) for x in cvrg])


def profile_matrix(sh, input, flank, binParams):
    """profileMatrix(input, flank, binParams) of rcp.R (one library call per sample)."""
    if not any(x.get("profile") is None for x in input):
        return input
    ln = _lengths(input[0]["coverage"])
    ln = ln[ln != 0]
    equal = bool(np.all(ln == ln[0])) if len(ln) else True
    stat = binParams.get("sumStat", "mean")
    for x in input:
        cvrg = x["coverage"]
        if equal:
            x["profile"] = bin_coverage_matrix(sh, cvrg, binParams["regionBinSize"], stat) \
                if binParams["regionBinSize"] != 0 else base_coverage_matrix(sh, cvrg)
            continue
        parts = rcp_parts(False, None, flank, binParams)
        x["profile"] = rcp_profile_rle(sh, cvrg, parts["where"], flank, parts["nBins"], parts["perBase"], stat,
                                       binParams.get("interpolation", "auto"), row_names=_names(cvrg))
    return input


# ---------------------------------------------------------------------------------------------
# The REFERENCE's own callers of binCoverageMatrix / baseCoverageMatrix, transliterated: with
# rcp.R dropped in, a maintainer who keeps R/profile.R's profileMatrix, and recoup()'s forced
# heatmap binning (R/recoup.R:659-714, which rcp.R does not replace), call the replacements above.
# R's cbind and rownames<- are modelled on the dimnames the shim returns.

def r_cbind(*mats):
    """cbind(...) of matrices (NULL arguments dropped): rownames from the first argument that has
    them; colnames the arguments' colnames, "" for an argument without; none if no argument has."""
    mats = [m for m in mats if m is not None]
    from tests.rmini.rmini import RArray
    vals = np.concatenate([np.asarray(m) for m in mats], axis=1)
    rn = next((m.rownames for m in mats if m.rownames is not None), None)
    cn = None
    if any(m.colnames is not None for m in mats):
        cn = []
        for m in mats:
            cn += list(m.colnames) if m.colnames is not None else [""] * m.shape[1]
    return RArray(vals, None if rn is None and cn is None else (rn, cn))


def r_set_rownames(m, names):
    """rownames(m) <- names."""
    from tests.rmini.rmini import RArray
    cn = m.colnames
    rn = None if names is None else list(names)
    return RArray(np.asarray(m), None if rn is None and cn is None else (rn, cn))


def ref_profile_matrix(sh, input, flank, binParams):
    """R/profile.R:1-98 as the reference wrote it, over rcp.R's binCoverageMatrix /
    baseCoverageMatrix."""
    if not any(x.get("profile") is None for x in input):
        return input
    ln = _lengths(input[0]["coverage"])
    ln = ln[ln != 0]
    equal = bool(np.all(ln == ln[0]))
    stat = binParams.get("sumStat", "mean")
    interp = binParams.get("interpolation", "auto")
    for x in input:
        cv = x["coverage"]
        if not equal:
            center = bin_coverage_matrix(sh, cv, binParams["regionBinSize"], stat, interp, flank, "center")
            r = np.asarray(flank, np.float64) / sum(flank)
            if binParams["flankBinSize"] != 0:
                left = None if flank[0] == 0 else bin_coverage_matrix(
                    sh, cv, int(np.round(2 * binParams["flankBinSize"] * r[0])), stat, interp, flank, "upstream")
                right = None if flank[1] == 0 else bin_coverage_matrix(
                    sh, cv, int(np.round(2 * binParams["flankBinSize"] * r[1])), stat, interp, flank, "downstream")
            else:
                left = None if flank[0] == 0 else base_coverage_matrix(sh, cv, flank, "upstream")
                right = None if flank[1] == 0 else base_coverage_matrix(sh, cv, flank, "downstream")
            x["profile"] = r_set_rownames(r_cbind(left, center, right), _names(cv))
        elif binParams["regionBinSize"] != 0:
            x["profile"] = bin_coverage_matrix(sh, cv, binParams["regionBinSize"], stat)
        else:
            x["profile"] = base_coverage_matrix(sh, cv)
    return input


def ref_forced_heatmap(sh, input, region, flank, binParams, customIsBase=False):
    """R/recoup.R:659-714: the heatmap profiles (helpInput[[n]]$profile), or None when the
    reference does not force binning.  A non-base region reaches :703, whose undefined
    forcedBinSize raises "object 'forcedBinSize' not found" after the center and upstream passes."""
    bp = dict(binParams)
    fbs = bp.get("forcedBinSize", (50, 200))
    if not (bp.get("forceHeatmapBinning", True) and (bp["regionBinSize"] == 0 or bp["flankBinSize"] == 0)):
        return None
    stat = bp.get("sumStat", "mean")
    out = []
    for x in input:
        if region in ("tss", "tes") or customIsBase:
            out.append(bin_coverage_matrix(sh, x["coverage"], fbs[1], stat))
            continue
        interp = bp.get("interpolation", "auto")
        bin_coverage_matrix(sh, x["coverage"], fbs[1], stat, interp, flank, "center")
        bin_coverage_matrix(sh, x["coverage"], fbs[0], stat, interp, flank, "upstream")
        raise NameError("object 'forcedBinSize' not found")
    return out
def profile_matrix_from_reads(sh, input, mask, flank, binParams, ignore_strand=True):
    """profileMatrixFromReads(input, mask, flank, binParams, ignore.strand)."""
    ln = mask.width
    equal = bool(np.all(ln == ln[0]))
    parts = rcp_parts(equal, int(ln[0]), flank, binParams)
    interp = "auto" if equal else binParams.get("interpolation", "auto")
    bin_args = [np.asarray(parts["where"], np.int32), np.asarray((0, 0) if flank is None else flank, np.int32),
                np.asarray(parts["nBins"], np.int32), np.asarray(parts["perBase"], np.int32),
                np.int32(STAT[binParams.get("sumStat", "mean")]), np.int32(INTERP[interp]), np.int32(0), 1.0]
    names = _rchar(mask.names)
    todo = [i for i, x in enumerate(input) if x.get("profile") is None]
    lv = list(dict.fromkeys(l for i in todo for l in input[i]["ranges"].seqlevels))
    rows = rcp_rows(mask, lv, ignore_strand)
    devices = rcp_devices()
    if len(devices) > 1:
        for i in todo:
            rs = rcp_read_set(sh, input[i]["ranges"], None, devices, lv, rows_of=lambda _lv: rows)
            res = sh.call("rcp_R_shards_profile", rs.ptr, *bin_args, names)
            rcp_free(sh, rs)
            input[i]["profile"] = res["profile"]
        return input
    read_args = [rcp_read_args(input[i]["ranges"], lv)[1] + [np.int32(-1)] for i in todo]
    res = sh.call("rcp_R_profile_reads", read_args, np.int32(devices[0]), *rcp_row_args(rows), *bin_args, names)
    for k, i in enumerate(todo):
        input[i]["profile"] = res[k]["profile"]
    return input
