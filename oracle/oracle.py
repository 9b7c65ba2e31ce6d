"""ctypes wrapper around the CPU ORACLE (``librcp_oracle.so``).

TEST INFRASTRUCTURE ONLY — imported by ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py``; never by the product package ``recoup_amd``.

Besides thin bindings, this module restates the reference's R-level orchestration of
the hot path so the tests can call it like the reference's own API:

* ``profile_matrix``     R/profile.R:1-98 (equal-length test on sample 1, per-base vs
                         binned, center/upstream/downstream + cbind)
* ``rna_merge``          R/coverage.R:115-121 (c(left, center, right), NULL if any NULL)
* ``profile_dimnames``   the dimnames of profileMatrix's matrix (rbind of a named list,
                         unlist of llply's bins, cbind + rownames<-)
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

WHERE = {"whole": 0, "center": 1, "upstream": 2, "downstream": 3}
INTERP = {"auto": 0, "spline": 1, "linear": 2, "neighborhood": 3}
STAT = {"mean": 0, "median": 1}
RNG = {"Rejection": 0, "Rounding": 1}

_i32p = ctypes.POINTER(ctypes.c_int32)
_i64p = ctypes.POINTER(ctypes.c_int64)
_i8p = ctypes.POINTER(ctypes.c_int8)
_u8p = ctypes.POINTER(ctypes.c_uint8)
_dp = ctypes.POINTER(ctypes.c_double)


class _ReadsIn(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int64), ("chrom", _i32p), ("start", _i32p), ("end", _i32p),
                ("strand", _i8p), ("n_chrom", ctypes.c_int32), ("seqlen", _i64p)]


class _MaskIn(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int32), ("seg_off", _i64p), ("seg_chrom", _i32p),
                ("seg_start", _i32p), ("seg_end", _i32p), ("seg_strand", _i8p)]


class _RowsIn(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int32), ("seg_off", _i64p), ("seg_chrom", _i32p), ("seg_start", _i32p),
                ("seg_end", _i32p), ("seg_strand", _i8p), ("seg_group", _i8p), ("group_is_list", _u8p)]


class _PartsIn(ctypes.Structure):
    _fields_ = [("n_parts", ctypes.c_int32), ("where", _i32p), ("n_bins", _i32p), ("per_base_width", _i32p),
                ("f1", ctypes.c_int32), ("f2", ctypes.c_int32), ("stat", ctypes.c_int32), ("interp", ctypes.c_int32),
                ("rng_kind", ctypes.c_int32), ("scale", ctypes.c_double)]


def build():
    """Compile the oracle with its own Makefile (gcc)."""
    import subprocess
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(HERE, "librcp_oracle.so")
        if not os.path.exists(path):
            build()
        L = ctypes.CDLL(path)
        L.orc_index_build.restype = ctypes.c_void_p
        L.orc_index_build.argtypes = [ctypes.POINTER(_ReadsIn), ctypes.c_int]
        L.orc_index_free.argtypes = [ctypes.c_void_p]
        L.orc_coverage.argtypes = [ctypes.c_void_p, ctypes.POINTER(_MaskIn), ctypes.c_int, ctypes.c_int,
                                   _i64p, _i32p, _u8p, _i64p]
        L.orc_split_vector.argtypes = [_dp, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                       ctypes.c_int, _dp, _i64p]
        L.orc_profile.argtypes = [ctypes.c_void_p, ctypes.POINTER(_MaskIn), ctypes.c_int, ctypes.c_double,
                                  ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                  ctypes.c_int, ctypes.c_int, ctypes.c_int, _dp, ctypes.c_int64, _u8p]
        L.orc_profile_rows.argtypes = [ctypes.c_void_p, ctypes.POINTER(_RowsIn), ctypes.POINTER(_PartsIn), ctypes.c_int,
                                       ctypes.c_int, _dp, _u8p]
        L.orc_set_seed.argtypes = [ctypes.c_uint32]
        L.orc_unif_rand.restype = ctypes.c_double
        L.orc_sample.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, _i32p]
        L.orc_spline.argtypes = [_dp, ctypes.c_int64, ctypes.c_int, _dp]
        _LIB = L
    return _LIB


def _p(a, t):
    return a.ctypes.data_as(t)


# ---------------------------------------------------------------- R RNG / spline
def set_seed(s):
    lib().orc_set_seed(ctypes.c_uint32(s & 0xFFFFFFFF))


def runif(k):
    return np.array([lib().orc_unif_rand() for _ in range(k)])


def sample_int(n, k, kind="Rejection"):
    out = np.zeros(max(k, 1), dtype=np.int32)
    rc = lib().orc_sample(n, k, RNG[kind], _p(out, _i32p))
    if rc:
        raise ValueError("cannot take a sample larger than the population")
    return out[:k]


def spline(y, n):
    y = np.ascontiguousarray(y, dtype=np.float64)
    out = np.zeros(n)
    lib().orc_spline(_p(y, _dp), len(y), n, _p(out, _dp))
    return out


def split_vector(x, n, interp="auto", stat="mean", kind="Rejection"):
    """splitVector(x, n, interp, stat) (R/util.R:15-85)."""
    x = np.ascontiguousarray(x, dtype=np.float64)
    out = np.zeros(max(n, len(x), 1))
    ol = np.zeros(1, dtype=np.int64)
    rc = lib().orc_split_vector(_p(x, _dp), len(x), n, INTERP[interp], STAT[stat], RNG[kind],
                                _p(out, _dp), _p(ol, _i64p))
    if rc:
        raise ValueError(f"splitVector: R would raise an error here (code {rc})")
    return out[:ol[0]]


# ---------------------------------------------------------------- reads / masks
class Index:
    """splitBySeqname of a flat read set (R/util.R:1-13) + optional strand filter."""

    def __init__(self, chrom, start, end, strand, seqlen, strand_filter=None):
        self._keep = [np.ascontiguousarray(chrom, dtype=np.int32),
                      np.ascontiguousarray(start, dtype=np.int32),
                      np.ascontiguousarray(end, dtype=np.int32),
                      np.ascontiguousarray(strand, dtype=np.int8),
                      np.ascontiguousarray(seqlen, dtype=np.int64)]
        c, s, e, st, sl = self._keep
        r = _ReadsIn(len(s), _p(c, _i32p), _p(s, _i32p), _p(e, _i32p), _p(st, _i8p), len(sl), _p(sl, _i64p))
        sf = -1 if strand_filter is None else {"+": 0, "-": 1, "*": 2}.get(strand_filter, strand_filter)
        self.h = lib().orc_index_build(ctypes.byref(r), sf)

    def __del__(self):
        if getattr(self, "h", None) and _LIB is not None:
            _LIB.orc_index_free(self.h)
            self.h = None


class Mask:
    """GRanges (one segment per element) or GRangesList (seg_off partitioning)."""

    def __init__(self, seg_off, chrom, start, end, strand):
        self.seg_off = np.ascontiguousarray(seg_off, dtype=np.int64)
        self.chrom = np.ascontiguousarray(chrom, dtype=np.int32)
        self.start = np.ascontiguousarray(start, dtype=np.int32)
        self.end = np.ascontiguousarray(end, dtype=np.int32)
        self.strand = np.ascontiguousarray(strand, dtype=np.int8)
        self.n = len(self.seg_off) - 1
        self.c = _MaskIn(self.n, _p(self.seg_off, _i64p), _p(self.chrom, _i32p), _p(self.start, _i32p),
                         _p(self.end, _i32p), _p(self.strand, _i8p))

    @classmethod
    def from_ranges(cls, chrom, start, end, strand):
        n = len(start)
        return cls(np.arange(n + 1), chrom, start, end, strand)


def coverage(index, mask, ignore_strand=True, nthreads=1):
    """calcCoverage -> list of int32 arrays (None for the reference's NULL)."""
    L = lib()
    ln = np.zeros(mask.n, dtype=np.int64)
    L.orc_coverage(index.h, ctypes.byref(mask.c), int(ignore_strand), nthreads, None, None, None, _p(ln, _i64p))
    off = np.zeros(mask.n + 1, dtype=np.int64)
    off[1:] = np.cumsum(ln)
    cov = np.zeros(max(int(off[-1]), 1), dtype=np.int32)
    valid = np.zeros(mask.n, dtype=np.uint8)
    ln2 = np.zeros(mask.n, dtype=np.int64)
    L.orc_coverage(index.h, ctypes.byref(mask.c), int(ignore_strand), nthreads, _p(off, _i64p),
                   _p(cov, _i32p), _p(valid, _u8p), _p(ln2, _i64p))
    return [cov[off[r]:off[r] + ln2[r]].copy() if valid[r] else None for r in range(mask.n)]


def profile_part(index, mask, n, ncol=None, where="whole", flank=(0, 0), interp="auto", stat="mean",
                 kind="Rejection", scale=1.0, ignore_strand=True, nthreads=1):
    """Fused reference dataflow per region: coverage -> slice -> splitVector -> row."""
    if ncol is None:
        ncol = n
    out = np.zeros((mask.n, ncol), dtype=np.float64, order="F")
    valid = np.zeros(mask.n, dtype=np.uint8)
    rc = lib().orc_profile(index.h, ctypes.byref(mask.c), int(ignore_strand), float(scale), WHERE[where],
                           int(flank[0]), int(flank[1]), int(n), INTERP[interp], STAT[stat], RNG[kind],
                           int(nthreads), out.ctypes.data_as(_dp), int(ncol), _p(valid, _u8p))
    if rc:
        raise ValueError(f"profile: R would raise an error here (code {rc})")
    return out, valid


def profile_rows(index, rows, bins, nthreads=1):
    """Rows of several mask elements (coverageRnaRef's c(left, exons, right), R/coverage.R:79-124)
    over several column parts (profileMatrix's cbind, R/profile.R:13-81), multithreaded over
    rows.  ``rows`` / ``bins`` are duck-typed like recoup_amd.engine.RowTable / Bins:
    rows.seg_off/chrom/start/end/strand/seg_group/group_is_list/ignore_strand, bins.where/
    n_bins/width/flank/stat/interp/rng_kind/scale.  Returns (R x n_cols F-order matrix, valid)."""
    keep = [np.ascontiguousarray(rows.seg_off, np.int64), np.ascontiguousarray(rows.chrom, np.int32),
            np.ascontiguousarray(rows.start, np.int32), np.ascontiguousarray(rows.end, np.int32),
            np.ascontiguousarray(rows.strand, np.int8),
            None if rows.seg_group is None else np.ascontiguousarray(rows.seg_group, np.int8),
            None if rows.group_is_list is None else np.ascontiguousarray(rows.group_is_list, np.uint8)]
    n = len(keep[0]) - 1
    ri = _RowsIn(n, _p(keep[0], _i64p), _p(keep[1], _i32p), _p(keep[2], _i32p), _p(keep[3], _i32p),
                 _p(keep[4], _i8p), None if keep[5] is None else _p(keep[5], _i8p),
                 None if keep[6] is None else _p(keep[6], _u8p))
    where = np.ascontiguousarray(bins.where, np.int32)
    nb = np.ascontiguousarray(bins.n_bins, np.int32)
    width = np.ascontiguousarray(bins.width, np.int32)
    pi = _PartsIn(len(nb), _p(where, _i32p), _p(nb, _i32p), _p(width, _i32p), int(bins.flank[0]), int(bins.flank[1]),
                  int(bins.stat), int(bins.interp), int(bins.rng_kind), float(bins.scale))
    ncol = int(sum(w if b == 0 else b for b, w in zip(nb, width)))
    out = np.zeros((n, ncol), dtype=np.float64, order="F")
    valid = np.zeros(n, dtype=np.uint8)
    rc = lib().orc_profile_rows(index.h, ctypes.byref(ri), ctypes.byref(pi), int(bool(rows.ignore_strand)),
                                int(nthreads), out.ctypes.data_as(_dp), _p(valid, _u8p))
    if rc:
        raise ValueError(f"profile_rows: R would raise an error here (code {rc})")
    return out, valid


# ---------------------------------------------------------------- R-level logic
def rna_merge(left, center, right):
    """coverage.R:115-121: c(le, ce, ri) per gene, NULL if any part is NULL."""
    out = []
    for le, ce, ri in zip(left, center, right):
        out.append(None if (le is None or ce is None or ri is None) else np.concatenate([le, ce, ri]))
    return out


def r_round(x):
    """R's round() (IEC 60559 half-to-even)."""
    return int(np.round(x))


def _bin_matrix(cov, n, stat, interp, flank=None, where="center", scale=1.0, kind="Rejection"):
    rows = []
    for x in cov:
        if x is None:
            v = np.zeros(n)
        else:
            v = x.astype(np.float64) * scale
            if flank is not None:
                L = len(v)
                if where == "center":
                    v = v[flank[0]:L - flank[1]]
                elif where == "upstream":
                    v = v[:flank[0]]
                else:
                    v = v[L - flank[1]:]
        rows.append(split_vector(v, n, interp, stat, kind))
    return _rbind(rows)


def _base_matrix(cov, flank=None, where="upstream", scale=1.0):
    if flank is None:
        size = next((len(x) for x in cov if x is not None), 0)
        rows = [np.zeros(size) if x is None else x.astype(np.float64) * scale for x in cov]
    else:
        size = flank[0] if where == "upstream" else flank[1]
        rows = []
        for x in cov:
            if x is None:
                rows.append(np.zeros(size))
            else:
                v = x.astype(np.float64) * scale
                rows.append(v[:flank[0]] if where == "upstream" else v[len(v) - flank[1]:])
    return _rbind(rows)


def _rbind(rows):
    ncol = max((len(r) for r in rows), default=0)
    out = np.zeros((len(rows), ncol))
    for i, r in enumerate(rows):
        if len(r):
            out[i] = np.resize(r, ncol)
    return out


def profile_matrix(covs, flank, bin_params, scales=None, kind="Rejection"):
    """profileMatrix (R/profile.R:1-98) over a list of per-sample coverage lists."""
    fbs = bin_params.get("flankBinSize", 0)
    rbs = bin_params.get("regionBinSize", 0)
    stat = bin_params.get("sumStat", "mean")
    interp = bin_params.get("interpolation", "auto")
    scales = scales or [1.0] * len(covs)
    lens = np.array([len(x) if x is not None else 0 for x in covs[0]])
    lens = lens[lens != 0]
    equal = bool(np.all(lens == lens[0])) if len(lens) else True
    out = []
    for cov, sc in zip(covs, scales):
        if not equal:
            center = _bin_matrix(cov, rbs, stat, interp, flank, "center", sc, kind)
            parts = []
            if fbs != 0:
                r = np.asarray(flank, dtype=float) / sum(flank)
                if flank[0] != 0:
                    parts.append(_bin_matrix(cov, r_round(2 * fbs * r[0]), stat, interp, flank, "upstream", sc, kind))
                parts.append(center)
                if flank[1] != 0:
                    parts.append(_bin_matrix(cov, r_round(2 * fbs * r[1]), stat, interp, flank, "downstream", sc, kind))
            else:
                if flank[0] != 0:
                    parts.append(_base_matrix(cov, flank, "upstream", sc))
                parts.append(center)
                if flank[1] != 0:
                    parts.append(_base_matrix(cov, flank, "downstream", sc))
            out.append(np.hstack(parts))
        else:
            if rbs != 0:
                out.append(_bin_matrix(cov, rbs, stat, interp, None, None, sc, kind))
            else:
                out.append(_base_matrix(cov, None, None, sc))
    return out


def bin_colnames(n, stat):
    """Names of a binned row, unlist(llply(split(x, f), stat)) (R/util.R:81-84, R/profile.R:208):
    split names the bins by the factor levels "1".."n"; llply hands a function given by NAME
    to plyr::each, whose one-function closure sets names(res) <- the function's name on a
    length-1 result, so unlist joins the two: "1.mean", "2.mean", ..."""
    return [f"{k}.{stat}" for k in range(1, int(n) + 1)]


def profile_dimnames(names, flank, bin_params, equal):
    """dimnames(input[[s]]$profile) after profileMatrix (R/profile.R:1-98) of a coverage list
    named ``names`` (None = unnamed): None, or (rownames, colnames).

    * equal lengths: the matrix is do.call("rbind", <list named like the coverage>) -- rownames
      = names (R/profile.R:112-115,159-162,198-208); binned rows bring bin_colnames, per-base
      rows (as.numeric of an Rle) none;
    * unequal: cbind(left, center, right) of slices mapped over 1:length(cvrg) (unnamed rows):
      colnames the parts' own, "" for a per-base flank; then rownames(...) <- names (:78-79)."""
    fbs = int(bin_params.get("flankBinSize", 0))
    rbs = int(bin_params.get("regionBinSize", 0))
    stat = bin_params.get("sumStat", "mean")
    rn = None if names is None else [str(x) for x in names]
    if equal:
        cn = bin_colnames(rbs, stat) if rbs != 0 else None
    else:
        f1, f2 = int(flank[0]), int(flank[1])
        r = np.asarray([f1, f2], dtype=float) / (f1 + f2)
        side = [bin_colnames(r_round(2 * fbs * r[k]), stat) if fbs != 0 else [""] * (f1, f2)[k]
                for k in (0, 1)]
        cn = (side[0] if f1 else []) + bin_colnames(rbs, stat) + (side[1] if f2 else [])
    return None if rn is None and cn is None else (rn, cn)


# ---------------------------------------------------------------- region windows
def promoters(start, end, strand, upstream, downstream):
    """GenomicRanges::promoters: '+'/'*' anchor at start, '-' anchor at end."""
    start = np.asarray(start, dtype=np.int64)
    end = np.asarray(end, dtype=np.int64)
    minus = np.asarray(strand) == 1
    s = np.where(minus, end - downstream + 1, start - upstream)
    e = np.where(minus, end + upstream, start + downstream - 1)
    return s, e


def resize(start, end, strand, width, fix="start"):
    """GenomicRanges::resize (fix relative to the transcription direction)."""
    start = np.asarray(start, dtype=np.int64)
    end = np.asarray(end, dtype=np.int64)
    width = np.broadcast_to(np.asarray(width, dtype=np.int64), start.shape)
    minus = np.asarray(strand) == 1
    keep_start = (~minus) if fix == "start" else minus
    s = np.where(keep_start, start, end - width + 1)
    e = np.where(keep_start, start + width - 1, end)
    return s, e


def flank_end(start, end, strand, width):
    """GenomicRanges::flank(x, width, start=FALSE, both=FALSE)."""
    start = np.asarray(start, dtype=np.int64)
    end = np.asarray(end, dtype=np.int64)
    minus = np.asarray(strand) == 1
    s = np.where(minus, start - width, end + 1)
    e = np.where(minus, start - 1, end + width)
    return s, e


def regional_ranges(start, end, strand, region, flank):
    """getRegionalRanges (R/ranges.R:67-91)."""
    f1, f2 = flank
    w = np.asarray(end, dtype=np.int64) - np.asarray(start, dtype=np.int64) + 1
    if region == "tss" or (region == "custom" and np.all(w == 1)):
        return promoters(start, end, strand, f1, f2)
    if region == "tes":
        s, e = resize(start, end, strand, 1, fix="end")
        return promoters(s, e, strand, f1, f2)
    s, e = promoters(start, end, strand, f1, 0)
    return resize(s, e, strand, w + f1 + f2, fix="start")
