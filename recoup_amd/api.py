"""The reference's R API for the coverage -> profile path, over the HIP engine.

Same names, argument meaning and result shapes as hjanime/recoup:

  calcCoverage(input, mask, strand, ignore_strand)        R/coverage.R:126-174
  coverageRef(input, genomeRanges, region, flank, ...)    R/coverage.R:1-77
  coverageRnaRef(input, genomeRanges, helperRanges, ...)  R/coverage.R:79-124
  profileMatrix(input, flank, binParams)                  R/profile.R:1-98
  binCoverageMatrix(cvrg, binSize, stat, interpolation, flank, where)   R/profile.R:153-212
  baseCoverageMatrix(cvrg, flank, where)                                R/profile.R:100-151
  calcLinearFactors(input) / normalizeLinear(input)       R/util.R:349-362, R/recoup.R:559-577

``input`` is a list of samples, each a dict with at least ``id``, ``name`` and ``ranges`` (a
``GRanges`` of reads) -- the reference's ``input`` list.  coverageRef / coverageRnaRef leave a
``DeviceCoverage`` in ``sample["coverage"]``: the reads stay indexed in HBM and the coverage
vectors are only materialised when asked for (``.to_list()``), because profileMatrix fuses
coverage and binning in one pass over the reads (no per-base vector ever reaches HBM).
Every call runs on the GPU through librecoup_amd.so; there is no CPU path.
"""
import os
import re

import numpy as np
import torch

from . import _lib
from .engine import Bins, Plan, ReadSet, RowTable, profile_rle
from .granges import GRanges, GRangesList, getFlankingRanges, getRegionalRanges


def _device(device):
    if device is not None:
        return int(device)
    return torch.cuda.current_device() if torch.cuda.is_available() else 0


def _first(x, default):
    if x is None:
        return default
    if isinstance(x, (list, tuple)):
        return x[0]
    return x


class CoverageList(list):
    """An R named list of coverage vectors (int32 numpy arrays or None for R's NULL)."""

    def __init__(self, items, names=None):
        super().__init__(items)
        self.names = None if names is None else list(names)

    def lengths(self):
        """R's lengths(): 0 for NULL elements."""
        return np.array([0 if x is None else len(x) for x in self], dtype=np.int64)


class Rle:
    """A run-length encoded integer vector (S4Vectors::Rle): ``values`` repeated ``lengths`` times."""

    __slots__ = ("values", "lengths")

    def __init__(self, values, lengths):
        self.values = np.asarray(values)
        self.lengths = np.asarray(lengths)

    def __len__(self):
        return int(self.lengths.sum())

    def decode(self):
        return np.repeat(self.values, self.lengths)

    def __mul__(self, k):  # Rle * numeric -> numeric Rle (normalize = "linear", R/recoup.R:559-577)
        return Rle(self.values * k, self.lengths)

    __rmul__ = __mul__

    def __repr__(self):
        return f"Rle({len(self)} positions in {len(self.values)} runs)"


class RMatrix(np.ndarray):
    """A numpy matrix that carries R's dimnames: ``rownames`` (region names) and ``colnames``."""

    def __new__(cls, a, rownames=None, colnames=None):
        obj = np.asarray(a).view(cls)
        obj.rownames = None if rownames is None else [str(x) for x in rownames]
        obj.colnames = None if colnames is None else list(colnames)
        return obj

    def __array_finalize__(self, obj):
        self.rownames = getattr(obj, "rownames", None)
        self.colnames = getattr(obj, "colnames", None)


_STAT_NAME = {0: "mean", 1: "median"}


def _colnames(bins):
    """The colnames R's rbind / cbind give a profile with these column parts: "<bin>.<stat>"
    per bin of a binned part -- unlist(llply(split(x, f), stat)) names each bin by its factor
    level and plyr::each names the length-1 statistic by the function's name (R/util.R:81-84,
    R/profile.R:208) -- and "" per column of a per-base part (as.numeric of an Rle has no
    names); None when no part is binned."""
    if not any(int(b) != 0 for b in bins.n_bins):
        return None
    stat = _STAT_NAME[bins.stat]
    out = []
    for b, w in zip(bins.n_bins, bins.width):
        out += [f"{k}.{stat}" for k in range(1, int(b) + 1)] if b else [""] * int(w)
    return out


# ------------------------------------------------------------------------------ reads
def _readset(reads, device, strand):
    """splitBySeqname + strand filter as a device index, cached on the GRanges object."""
    if isinstance(reads, ReadSet):
        if strand is not None:
            raise _lib.UnsupportedError(-4, "strand filtering needs the GRanges, not a prebuilt ReadSet")
        return reads, None
    if isinstance(reads, dict):  # a splitBySeqname() list: chromosome -> GRanges
        parts = [g for g in reads.values() if g is not None and len(g)]
        levels = list(dict.fromkeys(l for g in parts for l in g.seqlevels))
        reads = GRanges(np.concatenate([g.seqnames.astype(str) for g in parts]) if parts else np.array([], str),
                        np.concatenate([g.start for g in parts]) if parts else [],
                        np.concatenate([g.end for g in parts]) if parts else [],
                        np.concatenate([g.strand for g in parts]) if parts else [], seqlevels=levels,
                        seqlengths=_merge_seqlengths(parts, levels))
    if not isinstance(reads, GRanges):
        raise TypeError("input must be a GRanges of reads (or a per-chromosome dict of them)")
    cache = reads.__dict__.setdefault("_rcp_readsets", {})
    key = (device, strand)
    if key not in cache:
        if len(reads.seqlevels) == 0:
            reads = GRanges(np.array(["."]), [1], [0])[np.zeros(0, dtype=np.int64)]
        cache[key] = ReadSet(reads.seqcodes, reads.start.astype(np.int32), reads.end.astype(np.int32), reads.strand,
                             reads.seqlengths, device=device, strand_filter=strand)
    return cache[key], reads.seqlevels


def _merge_seqlengths(parts, levels):
    sl = {}
    for g in parts:
        for l, v in zip(g.seqlevels, g.seqlengths):
            if v >= 0:
                sl[l] = int(v)
    return sl


def _rows_from_mask(mask, levels, ignore_strand):
    """RowTable for a GRanges (one range per row) or GRangesList (one element per row)."""
    if isinstance(mask, GRangesList):
        flat = mask.flat
        chrom = flat.codes_in(levels) if levels is not None else flat.seqcodes
        n = len(flat)
        return RowTable(mask.offsets, chrom, _i32(flat.start), _i32(flat.end), flat.strand,
                        seg_group=np.zeros(n, np.int8), group_is_list=np.array([1, 0, 0, 0], np.uint8),
                        ignore_strand=ignore_strand, names=mask.names)
    if isinstance(mask, GRanges):
        chrom = mask.codes_in(levels) if levels is not None else mask.seqcodes
        return RowTable.from_ranges(chrom, _i32(mask.start), _i32(mask.end), mask.strand,
                                    ignore_strand=ignore_strand, names=mask.names)
    raise TypeError("The mask argument must be a GRanges or GRangesList object")


def _i32(a):
    a = np.asarray(a)
    if a.size and (a.min() < -(2 ** 31) or a.max() >= 2 ** 31):
        raise _lib.UnsupportedError(-4, "coordinates beyond int32")
    return a.astype(np.int32)


class DeviceCoverage:
    """The coverage list of one sample over one mask, kept as (device reads, row table).

    ``len`` / ``names`` / ``lengths()`` / ``to_list()`` answer like the R list of Rle the
    reference stores in ``input[[s]]$coverage``; profileMatrix bins it on the GPU directly.
    ``scale`` is the normalisation factor applied to the coverage (normalize = "linear")."""

    def __init__(self, readset, rows, names=None, scale=1.0):
        self.readset = readset
        self.rows = rows
        self.names = None if names is None else list(names)
        self.scale = float(scale)
        self._len = None
        self._valid = None

    def __len__(self):
        return self.rows.n_rows

    def _plan(self):
        return Plan(self.readset, self.rows, None)

    def valid(self):
        if self._valid is None:
            p = self._plan()
            self._valid = p.validity()
            self._len = p.row_lengths()
        return self._valid

    def lengths(self):
        """R's lengths(cov): the row's length, 0 where the coverage is NULL."""
        v = self.valid()
        return np.where(v, self._len, 0)

    def to_list(self, rle=False):
        """Materialise the per-region coverage vectors (calcCoverage's return value); with
        ``rle`` as ``Rle`` objects run-length encoded on the GPU."""
        cov = self._plan().coverage(rle=rle)
        if rle:
            cov = [None if x is None else Rle(x[0] * self.scale if self.scale != 1.0 else x[0], x[1]) for x in cov]
        elif self.scale != 1.0:
            cov = [None if x is None else x.astype(np.float64) * self.scale for x in cov]
        return CoverageList(cov, self.names)

    def scaled(self, factor):
        return DeviceCoverage(self.readset, self.rows, self.names, self.scale * float(factor))


# ------------------------------------------------------------------------------ coverage
def _bam_reads(path):
    """calcCoverage's file input (R/coverage.R:127-140): a BAM path is read by coverageFromBam
    (:228-295), one region at a time, as every mapped alignment overlapping it
    (``ScanBamParam(which=)``, spliceAction "keep": the alignment's reference span).  Reading
    the whole file once (readBam, "keep") and locating each region's reads on the GPU gives
    the same reads per region; the BAM header's lengths are the seqlengths."""
    path = os.fspath(path)
    if not os.path.exists(path):
        raise ValueError("The input argument must be a GenomicRanges object or a valid BAM/BigWig file "
                         "or a list of GenomicRanges")
    if re.search(r"\.bam$", path, re.IGNORECASE) is None:
        if re.search(r"\.(bigwig|bw|wig|bg)$", path, re.IGNORECASE):
            raise _lib.UnsupportedError(-4, "BigWig input (coverageFromBigWig) is not on the GPU path")
        raise ValueError("The input argument must be a GenomicRanges object or a valid BAM/BigWig file "
                         "or a list of GenomicRanges")
    return readBam(path, "keep")


def _sample_reads(s, strand, ignore_strand):
    """A sample's reads for coverageRef / coverageRnaRef: ``ranges`` when present, else its
    ``file`` -- the reference passes ``input[[n]]$file`` to calcCoverage (coverage.R:35-39,
    58-62, 93-96), whose BAM branch skips the strand filter (:141) and never reads
    ``ignore.strand`` (coverageFromBam takes every overlapping alignment)."""
    if s.get("ranges") is not None:
        return s["ranges"], strand, ignore_strand
    if s.get("file") is not None:
        return _bam_reads(s["file"]), None, True
    raise ValueError(f"sample {s.get('id')!r} has neither ranges nor a file")


def calcCoverage(input, mask, strand=None, ignore_strand=True, device=None, rc=None, rle=False):
    """R/coverage.R:126-174: one coverage vector per mask element (None = R's NULL); with
    ``rle`` the elements are ``Rle`` objects, the form the reference returns.  ``input`` may
    also be a BAM file path (coverageFromBam semantics: no strand filter, strand ignored)."""
    if isinstance(input, (str, os.PathLike)):
        input, strand, ignore_strand = _bam_reads(input), None, True
    dev = _device(device)
    rs, levels = _readset(input, dev, strand)
    rows = _rows_from_mask(mask, levels, ignore_strand)
    return DeviceCoverage(rs, rows, mask.names).to_list(rle=rle)


def _strand_params(sp):
    sp = sp or {}
    return sp.get("strand"), bool(sp.get("ignoreStrand", True))


def _needs(input, key):
    """The reference recomputes only when some sample lacks the slot (coverage.R:4-6)."""
    return any(s.get(key) is None for s in input)


def coverageRef(input, genomeRanges, region="tss", flank=(2000, 2000), strandedParams=None, bamParams=None,
                rc=None, device=None):
    """R/coverage.R:1-77 (coverageBaseRef / coverageAreaRef share calcCoverage)."""
    if not _needs(input, "coverage"):
        return input
    region = _first(region, "tss")
    main = getRegionalRanges(genomeRanges, region, flank)
    strand, ign = _strand_params(strandedParams)
    dev = _device(device)
    for s in input:
        reads, st, ig = _sample_reads(s, strand, ign)
        rs, levels = _readset(reads, dev, st)
        s["coverage"] = DeviceCoverage(rs, _rows_from_mask(main, levels, ig), genomeRanges.names)
    return input


def _rna_rows(genomeRanges, helperRanges, flank, levels, ignore_strand):
    """Rows c(left flank, exons..., right flank) per gene (coverage.R:84-120), groups 0 / 1 / 2."""
    f1, f2 = int(flank[0]), int(flank[1])
    left = getFlankingRanges(helperRanges, 1 if f1 == 0 else f1, "upstream")
    right = getFlankingRanges(helperRanges, 1 if f1 == 0 else f2, "downstream")  # the reference tests flank[1]
    G = len(genomeRanges)
    if len(helperRanges) != G:
        raise _lib.SemanticError(-5, "helperRanges and genomeRanges differ in length")
    ex = genomeRanges.flat
    n_ex = np.diff(genomeRanges.offsets)
    seg_off = np.zeros(G + 1, dtype=np.int64)
    seg_off[1:] = np.cumsum(n_ex + 2)
    n = int(seg_off[-1])
    first = seg_off[:-1]
    last = seg_off[1:] - 1
    is_ex = np.ones(n, dtype=bool)
    is_ex[first] = False
    is_ex[last] = False
    chrom = np.empty(n, np.int32)
    start = np.empty(n, np.int64)
    end = np.empty(n, np.int64)
    strand = np.empty(n, np.int8)
    group = np.ones(n, np.int8)
    chrom[first], start[first], end[first], strand[first], group[first] = \
        left.codes_in(levels), left.start, left.end, left.strand, 0
    chrom[last], start[last], end[last], strand[last], group[last] = \
        right.codes_in(levels), right.start, right.end, right.strand, 2
    chrom[is_ex], start[is_ex], end[is_ex], strand[is_ex] = ex.codes_in(levels), ex.start, ex.end, ex.strand
    return RowTable(seg_off, chrom, _i32(start), _i32(end), strand, seg_group=group,
                    group_is_list=np.array([0, 1, 0, 0], np.uint8), ignore_strand=ignore_strand,
                    names=genomeRanges.names)


def coverageRnaRef(input, genomeRanges, helperRanges, flank=(2000, 2000), strandedParams=None, bamParams=None,
                   rc=None, device=None):
    """R/coverage.R:79-124: exon-concatenated gene coverage with gene flanks, NULL if any part is NULL."""
    if not _needs(input, "coverage"):
        return input
    strand, ign = _strand_params(strandedParams)
    dev = _device(device)
    for s in input:
        reads, st, ig = _sample_reads(s, strand, ign)
        rs, levels = _readset(reads, dev, st)
        s["coverage"] = DeviceCoverage(rs, _rna_rows(genomeRanges, helperRanges, flank, levels, ig),
                                       genomeRanges.names)
    return input


# ------------------------------------------------------------------------------ profile
def _as_coverage(cvrg):
    """A DeviceCoverage (reads in HBM + row table: the fused pass), or a host coverage list --
    the reference's own ``$coverage`` object: a list of Rle / vectors / None (profiled from its
    runs by rcp_profile_rle)."""
    if isinstance(cvrg, DeviceCoverage):
        return cvrg
    if isinstance(cvrg, (list, tuple)):
        return cvrg if isinstance(cvrg, CoverageList) else CoverageList(list(cvrg), getattr(cvrg, "names", None))
    raise TypeError("a coverage must be a DeviceCoverage or a list of Rle / vectors / None")


def _run(cv, bins, device=None, named=True):
    """``named``: rows named by the coverage list (rbind of cmclapply(cvrg, ...)); False for the
    flank / center slices, mapped over 1:length(cvrg) (R/profile.R:125-141,164-189)."""
    if isinstance(cv, DeviceCoverage):
        plan = Plan(cv.readset, cv.rows, bins)
        mat, _ = plan.run()
    else:
        mat, _ = profile_rle(cv, bins, device=_device(device))
    return RMatrix(mat, cv.names if named else None, _colnames(bins))


def _scale_of(cv):
    return cv.scale if isinstance(cv, DeviceCoverage) else 1.0  # a host list holds scaled values


def binCoverageMatrix(cvrg, binSize=1000, stat="mean", interpolation="auto", flank=None, where="center", rc=None,
                      device=None):
    """R/profile.R:153-212: splitVector of each (sliced) coverage vector into binSize bins.
    ``cvrg``: a DeviceCoverage or the reference's list of Rle (None = NULL)."""
    cv = _as_coverage(cvrg)
    stat = str(_first(stat, "mean")).lower()
    interpolation = _first(interpolation, "auto")
    where = _first(where, "center")
    if flank is None:
        bins = Bins([("whole", int(binSize))], stat=stat, interp=interpolation, scale=_scale_of(cv))
    else:
        bins = Bins([(where, int(binSize))], flank=flank, stat=stat, interp=interpolation, scale=_scale_of(cv))
    return _run(cv, bins, device, named=flank is None)


def _base_size(cv):
    ln = cv.lengths()
    nz = ln[ln > 0]
    # baseCoverageMatrix sizes NULL rows from element 1, else the first non-NULL element
    return int(ln[0]) if len(ln) and ln[0] > 0 else (int(nz[0]) if len(nz) else 0)


def baseCoverageMatrix(cvrg, flank=None, where="upstream", rc=None, device=None):
    """R/profile.R:100-151: per-base coverage rows (NULL -> zeros); ``cvrg`` as for
    binCoverageMatrix."""
    cv = _as_coverage(cvrg)
    where = _first(where, "upstream")
    if flank is None:
        bins = Bins([("whole", 0, _base_size(cv))], scale=_scale_of(cv))
    else:
        size = int(flank[0]) if where == "upstream" else int(flank[1])
        bins = Bins([(where, 0, size)], flank=flank, scale=_scale_of(cv))
    return _run(cv, bins, device, named=flank is None)


def _profile_bins(binParams, flank, equal, size):
    """The column parts profileMatrix assembles (profile.R:13-96), fused into one plan."""
    fbs = int(binParams.get("flankBinSize", 0))
    rbs = int(binParams.get("regionBinSize", 0))
    stat = str(_first(binParams.get("sumStat"), "mean")).lower()
    interp = _first(binParams.get("interpolation"), "auto")
    if equal:
        if rbs != 0:  # the equal-length branch leaves interpolation at its default (profile.R:87-89)
            return Bins([("whole", rbs)], stat=stat, interp="auto")
        return Bins([("whole", 0, size)])
    f1, f2 = int(flank[0]), int(flank[1])
    parts = []
    if fbs != 0:
        r = np.asarray([f1, f2], dtype=float) / (f1 + f2)
        nb = [int(np.round(2 * fbs * r[k])) for k in (0, 1)]
        if any(f and b == 0 for f, b in zip((f1, f2), nb)):
            # binCoverageMatrix(binSize = 0) stops in splitVector's sample() (R/util.R:74-79)
            raise _lib.SemanticError(-5, "invalid 'size' argument (a flank rounds to 0 bins)")
        if f1:
            parts.append(("upstream", nb[0]))
        parts.append(("center", rbs))
        if f2:
            parts.append(("downstream", nb[1]))
    else:
        if f1:
            parts.append(("upstream", 0, f1))
        parts.append(("center", rbs))
        if f2:
            parts.append(("downstream", 0, f2))
    return Bins(parts, flank=(f1, f2), stat=stat, interp=interp)


def _profile_pass(cv, bins, keep_on_device=False, device=None):
    """One fused pass over a coverage: (R x n_cols host matrix, device (n_cols, R) view or None).
    A DeviceCoverage runs the read plan (padded column stride); a host list the Rle path."""
    if isinstance(cv, DeviceCoverage):
        bins.scale = cv.scale
        plan = Plan(cv.readset, cv.rows, bins, out_ld="padded")
        out = plan.empty_output()
        valid = torch.empty(max(plan.n_rows, 1), dtype=torch.uint8, device=out.device)
        plan.execute(out, valid)
        plan.status()
        return out[:, :plan.n_rows].cpu().numpy().T, (out[:, :plan.n_rows] if keep_on_device else None)
    mat, _ = profile_rle(cv, bins, device=_device(device))
    return mat, (torch.from_numpy(np.ascontiguousarray(mat.T)).to(f"cuda:{_device(device)}")
                 if keep_on_device else None)


def profileMatrix(input, flank, binParams, rc=None, keep_on_device=False):
    """R/profile.R:1-98: per-sample R x B double matrix in ``sample["profile"]``.

    The equal-length test uses the first sample's non-NULL lengths only (profile.R:6-10).
    With ``keep_on_device`` the column-major float64 matrix also stays in HBM as
    ``sample["profile_device"]`` (shape (B, R) in torch terms)."""
    if not _needs(input, "profile"):
        return input
    cvs = [_as_coverage(s["coverage"]) for s in input]
    ln = cvs[0].lengths()
    ln = ln[ln != 0]
    equal = bool(np.all(ln == ln[0])) if len(ln) else True
    for s, cv in zip(input, cvs):
        bins = _profile_bins(binParams, flank, equal, _base_size(cv) if equal else 0)
        mat, dev = _profile_pass(cv, bins, keep_on_device)
        s["profile"] = RMatrix(mat, cv.names, _colnames(bins))
        if keep_on_device:
            s["profile_device"] = dev
    return input


def recoupProfiles(input, genomeRanges, region, flank, binParams, keep_on_device=False):
    """The profile steps of recoup() over coverages already in ``input``: the forced
    regionBinSize (R/recoup.R:579-596), profileMatrix (:597) and the forced heatmap binning
    pass (:659-714), computed in ONE device pass per sample when both agree on the statistic
    and interpolation (the plan's column parts are the profile's followed by the heatmap's).
    Leaves ``sample["profile"]`` and, when the reference computes it, ``sample["heatmap"]``.

    As in the reference, the heatmap pass of a non-base region (genebody / wide custom) fails:
    R/recoup.R:703 reads the undefined ``forcedBinSize[1]`` -> SemanticError."""
    bp = dict(binParams)
    f1, f2 = int(flank[0]), int(flank[1])
    custom_is_base = region == "custom" and bool(np.all(genomeRanges.width == 1))
    must_bin = region == "genebody" or (region == "custom" and not bool(np.all(genomeRanges.width == genomeRanges.width[0])))
    if must_bin and int(bp.get("regionBinSize", 0)) == 0:
        bp["regionBinSize"] = 1000  # R/recoup.R:590-596
    forced = bool(bp.get("forceHeatmapBinning", True)) and (int(bp.get("regionBinSize", 0)) == 0 or
                                                              int(bp.get("flankBinSize", 0)) == 0)
    base_region = region in ("tss", "tes") or custom_is_base
    if forced and not base_region:
        raise _lib.SemanticError(-5, "recoup.R:703: object 'forcedBinSize' not found (the reference's forced "
                                     "heatmap binning of a non-base region)")
    fbs = bp.get("forcedBinSize", (50, 200))
    cvs = [_as_coverage(s["coverage"]) for s in input]
    ln = cvs[0].lengths()
    ln = ln[ln != 0]
    equal = bool(np.all(ln == ln[0])) if len(ln) else True
    stat = str(_first(bp.get("sumStat"), "mean")).lower()
    for s, cv in zip(input, cvs):
        prof = _profile_bins(bp, flank, equal, _base_size(cv) if equal else 0)
        parts = list(prof.parts)
        heat = None
        if forced:
            # binCoverageMatrix(coverage, binSize = forcedBinSize[2], stat) with its default
            # interpolation "auto" (R/recoup.R:664-668)
            heat = Bins([("whole", int(fbs[1]))], stat=stat, interp="auto")
        fuse = heat is not None and prof.interp == heat.interp and prof.stat == heat.stat
        bins = Bins(parts + (heat.parts if fuse else []), flank=(f1, f2), stat=prof.stat, interp=prof.interp)
        full, dev = _profile_pass(cv, bins, keep_on_device)
        npc = prof.n_cols
        s["profile"] = RMatrix(full[:, :npc], cv.names, _colnames(prof))
        if keep_on_device:
            s["profile_device"] = dev
        if heat is not None:
            if fuse:
                s["heatmap"] = RMatrix(full[:, npc:], cv.names, _colnames(heat))
            else:
                heat.scale = _scale_of(cv)
                s["heatmap"] = _run(cv, heat)
    return input


# ------------------------------------------------------------------------------ normalisation
def calcLinearFactors(input, preprocessParams=None):
    """R/util.R:349-362: min(libsize) / libsize ("linear", "downsample") or sampleTo / libsize
    ("sampleto") per sample, libsize = number of reads."""
    if any(s.get("ranges") is None for s in input):
        raise _lib.SemanticError(-5, "Please provide input reads before calculation normalization factors")
    pp = preprocessParams or {"normalize": "linear"}
    lib = np.array([len(s["ranges"]) for s in input], dtype=np.float64)
    if pp.get("normalize") in ("linear", "downsample"):
        return lib.min() / lib
    if pp.get("normalize") == "sampleto":
        return float(pp["sampleTo"]) / lib
    raise _lib.SemanticError(-5, f"no linear factors for normalize = {pp.get('normalize')!r}")


def normalizeLinear(input):
    """R/recoup.R:559-577 (normalize = "linear"): scale each sample's coverage."""
    f = calcLinearFactors(input)
    for s, k in zip(input, f):
        if k == 1:
            continue
        cv = s.get("coverage")
        if isinstance(cv, DeviceCoverage):
            s["coverage"] = cv.scaled(k)
        elif cv is not None:
            s["coverage"] = CoverageList([None if x is None else x * k for x in cv], cv.names)
    return input


# ------------------------------------------------------------------------------ ingest
SPLICE = {"keep": 0, "remove": 1, "split": 2}


def readBam(bam, spliceAction="keep", spliceRemoveQ=0.75, threads=8):
    """readBam (R/ranges.R:120-146): the mapped alignments of a BAM file as a GRanges of
    reads (BGZF inflated on ``threads`` host threads by librecoup_amd.so)."""
    import ctypes
    L = _lib.lib()
    h = ctypes.c_void_p()
    _lib.check(L.rcp_bam_read(str(bam).encode(), SPLICE[_first(spliceAction, "keep")], float(spliceRemoveQ),
                              int(threads), ctypes.byref(h)))
    try:
        n = ctypes.c_int64()
        nref = ctypes.c_int32()
        nal = ctypes.c_int64()
        _lib.check(L.rcp_bam_info(h, ctypes.byref(n), ctypes.byref(nref), ctypes.byref(nal)))
        names = [L.rcp_bam_ref_name(h, i).decode() for i in range(nref.value)]
        ref_len = np.zeros(max(nref.value, 1), np.int64)
        chrom = np.zeros(n.value, np.int32)
        start = np.zeros(n.value, np.int32)
        end = np.zeros(n.value, np.int32)
        strand = np.zeros(n.value, np.int8)
        _lib.check(L.rcp_bam_copy(h, _lib.cptr(ref_len, _lib._i64p), _lib.cptr(chrom, _lib._i32p),
                                  _lib.cptr(start, _lib._i32p), _lib.cptr(end, _lib._i32p),
                                  _lib.cptr(strand, _lib._i8p)))
    finally:
        L.rcp_bam_free(h)
    return GRanges(chrom, start, end, strand, seqlevels=names, seqlengths=ref_len[:len(names)])


class RRng:
    """R's RNG after ``set.seed(seed)`` (Mersenne-Twister, ``sample.kind`` Rejection or Rounding)."""

    def __init__(self, seed, kind="Rejection"):
        import ctypes
        self._h = ctypes.c_void_p()
        _lib.check(_lib.lib().rcp_rng_create(int(seed) & 0xFFFFFFFF, {"Rejection": 0, "Rounding": 1}[kind],
                                             ctypes.byref(self._h)))

    def runif(self, k):
        out = np.zeros(max(int(k), 1))
        _lib.check(_lib.lib().rcp_rng_unif(self._h, int(k), _lib.cptr(out, _lib._dp)))
        return out[:k]

    def sample_sorted(self, n, k):
        """``sort(sample(n, k))`` (1-based)."""
        out = np.zeros(max(int(k), 1), dtype=np.int64)
        _lib.check(_lib.lib().rcp_rng_sample_sorted(self._h, int(n), int(k), _lib.cptr(out, _lib._i64p)))
        return out[:k]

    def __del__(self):
        try:
            _lib.lib().rcp_rng_free(self._h)
        except Exception:
            pass


def preprocessRanges(input, preprocessParams=None, bamParams=None, rc=None):
    """R/ranges.R:1-62: read each sample's BAM (``file``, when ``ranges`` is missing) and apply
    normalize = "downsample" (every sample down to the smallest library) or "sampleto"
    (every sample to ``sampleTo`` reads): ``set.seed(seed)`` once, then per sample
    ``ranges[sort(sample(libsize, size))]``.  "none" / "linear" only read."""
    pp = {"normalize": "none", "sampleTo": 1e6, "spliceAction": "split", "spliceRemoveQ": 0.75, "seed": 42}
    pp.update(preprocessParams or {})
    if not _needs(input, "ranges"):
        return input
    for s in input:
        if s.get("ranges") is None:
            fmt = str(s.get("format", "bam")).lower()
            if fmt != "bam":
                raise _lib.UnsupportedError(-4, f"reading {fmt} input is outside this build (BAM only)")
            s["ranges"] = readBam(s["file"], _first(pp["spliceAction"], "split"), pp["spliceRemoveQ"])
    norm = _first(pp["normalize"], "none")
    if norm in ("downsample", "sampleto"):
        libs = [len(s["ranges"]) for s in input]
        size = min(libs) if norm == "downsample" else int(pp["sampleTo"])
        rng = RRng(int(pp["seed"]))
        for s, n in zip(input, libs):
            idx = rng.sample_sorted(n, size) - 1
            s["ranges"] = s["ranges"][idx]
    return input
