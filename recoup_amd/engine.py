"""Device-resident read sets and profile plans (thin RAII wrappers over the C ABI).

``ReadSet``  -- splitBySeqname (R/util.R:1-13) + strand filter (R/coverage.R:141-144) as a
               GPU index: reads sorted by (chromosome, strand, start) with a prefix-max-of-end
               array, held in HBM for the lifetime of the object.
``RowTable`` -- the mask side: one row per region (GRanges element) or per coverageRnaRef
               gene (upstream flank, exon list, downstream flank).
``Plan``     -- one coverage -> profile pass (R/coverage.R:176-226 fused with
               R/profile.R:100-212 and R/util.R:15-85) ready to execute on a HIP stream.
"""
import ctypes

import numpy as np
import torch

from . import _lib
from ._lib import check, cptr, ptr

STRAND = {"+": 0, "-": 1, "*": 2}
STAT = {"mean": 0, "median": 1}
INTERP = {"auto": 0, "spline": 1, "linear": 2, "neighborhood": 3}
RNG = {"Rejection": 0, "Rounding": 1}
KERNEL = {"auto": 0, "general": 1, "lean_any": 2, "rows": 3, "lean": 4, "bins": 5}


def _stream(device, stream):
    if stream is None:
        return _lib.stream_handle(device)
    if isinstance(stream, torch.cuda.Stream):
        return ctypes.c_void_p(stream.cuda_stream)
    return ctypes.c_void_p(stream)


def _chrom_runs(chrom):
    """(run_values int32, run_lengths int64) when ``chrom`` (or ``end``) is given as the runs of
    an R Rle (seqnames(x), width(x)), else None."""
    if isinstance(chrom, tuple) and len(chrom) == 2:
        v = np.ascontiguousarray(chrom[0], dtype=np.int32)
        n = np.ascontiguousarray(chrom[1], dtype=np.int64)
        if v.shape != n.shape:
            raise ValueError("runs: values and lengths differ in length")
        return v, n
    return None


def _reads_desc(n, keep, runs, seql, device, on_dev, sf, wruns=None):
    d = _lib.ReadsDesc(n, ptr(keep[0]) if keep[0] is not None else None, ptr(keep[1]),
                       ptr(keep[2]) if keep[2] is not None else None, ptr(keep[3]),
                       len(seql), cptr(seql, _lib._i64p), device, on_dev, sf)
    if runs is not None:
        d.n_chrom_runs = len(runs[0])
        d.chrom_run_value = cptr(runs[0], _lib._i32p)
        d.chrom_run_length = cptr(runs[1], _lib._i64p)
    if wruns is not None:
        d.n_width_runs = len(wruns[0])
        d.width_run_value = cptr(wruns[0], _lib._i32p)
        d.width_run_length = cptr(wruns[1], _lib._i64p)
    d._keep = (keep, runs, wruns)  # the arrays outlive the call
    return d


class ReadSet:
    """Reads of one sample, resident on one GPU.

    ``chrom``/``start``/``end``/``strand`` may be numpy arrays (uploaded) or torch CUDA
    tensors already on ``device`` (adopted, no host round trip).  ``seqlengths`` has one
    entry per chromosome code, -1 for NA.
    """

    def __init__(self, chrom, start, end, strand, seqlengths, device=0, strand_filter=None, stream=None):
        """``chrom`` is one code per read, or the runs of R's ``seqnames(x)`` Rle as a tuple
        ``(run_values, run_lengths)`` (expanded on the GPU, never copied per read); likewise
        ``end`` is one end per read, or the runs of ``width(x)`` as a tuple ``(run_values,
        run_lengths)`` (end = start + width - 1 formed on the GPU)."""
        lib = _lib.lib()
        if _lib.device_count() == 0:
            raise _lib.RcpError(-6, "no GPU visible: recoup_amd runs only on the GPU")
        self.device = int(device)
        self.seqlengths = np.ascontiguousarray(seqlengths, dtype=np.int64)
        on_dev = isinstance(start, torch.Tensor)
        runs = _chrom_runs(chrom)
        wruns = _chrom_runs(end)
        if on_dev:
            keep = ([None if runs else chrom.contiguous(), start.contiguous(), None if wruns else end.contiguous(),
                     strand.contiguous()])
            for t, dt in zip(keep, (torch.int32, torch.int32, torch.int32, torch.int8)):
                if t is not None and (t.dtype != dt or t.device.type != "cuda"):
                    raise TypeError("device reads must be int32/int32/int32/int8 CUDA tensors")
        else:
            keep = [None if runs else np.ascontiguousarray(chrom, dtype=np.int32),
                    np.ascontiguousarray(start, dtype=np.int32),
                    None if wruns else np.ascontiguousarray(end, dtype=np.int32),
                    np.ascontiguousarray(strand, dtype=np.int8)]
        n = int(keep[1].shape[0])
        sf = -1 if strand_filter is None else STRAND.get(strand_filter, strand_filter)
        d = _reads_desc(n, keep, runs, self.seqlengths, self.device, int(on_dev), int(sf), wruns)
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            check(lib.rcp_readset_create(ctypes.byref(d), _stream(self.device, stream), ctypes.byref(h)))
        self.h = h
        self._stream_off = None
        nk = ctypes.c_int64()
        check(lib.rcp_readset_info(self.h, ctypes.byref(nk), None))
        self.n = nk.value

    @classmethod
    def multi(cls, chrom, start, end, strand, seqlengths, devices, strand_filter=None):
        """rcp_readset_create_multi: one readset of the same host reads on each of ``devices``
        (one host thread per GPU), for profile_multi."""
        lib = _lib.lib()
        seql = np.ascontiguousarray(seqlengths, dtype=np.int64)
        runs = _chrom_runs(chrom)
        wruns = _chrom_runs(end)
        keep = [None if runs else np.ascontiguousarray(chrom, dtype=np.int32),
                np.ascontiguousarray(start, dtype=np.int32),
                None if wruns else np.ascontiguousarray(end, dtype=np.int32),
                np.ascontiguousarray(strand, dtype=np.int8)]
        sf = -1 if strand_filter is None else STRAND.get(strand_filter, strand_filter)
        d = _reads_desc(int(keep[1].shape[0]), keep, runs, seql, 0, 0, int(sf), wruns)
        dev = np.ascontiguousarray(devices, dtype=np.int32)
        hs = (ctypes.c_void_p * len(dev))()
        check(lib.rcp_readset_create_multi(ctypes.byref(d), cptr(dev, _lib._i32p), len(dev), hs))
        out = []
        for h, dv in zip(hs, dev):
            rs = cls.__new__(cls)
            rs.device, rs.seqlengths, rs.h = int(dv), seql, ctypes.c_void_p(h)
            rs._stream_off = None
            nk = ctypes.c_int64()
            check(lib.rcp_readset_info(rs.h, ctypes.byref(nk), None))
            rs.n = nk.value
            out.append(rs)
        return out

    @property
    def stream_off(self):
        """Start of each (chromosome, strand) stream of the strand-split layout, [3 * n_chrom + 1]
        (rcp_readset_info; the library builds that layout on its first use, so a readset only
        ever used with ignore.strand = TRUE rows never pays for it)."""
        if self._stream_off is None:
            so = np.zeros(3 * len(self.seqlengths) + 1, dtype=np.int64)
            nk = ctypes.c_int64()
            with torch.cuda.device(self.device):
                check(_lib.lib().rcp_readset_info(self.h, ctypes.byref(nk), cptr(so, _lib._i64p)))
            self._stream_off = so
        return self._stream_off

    @property
    def chrom_has_reads(self):
        so = self.stream_off
        return np.array([so[3 * c + 3] > so[3 * c] for c in range(len(self.seqlengths))])

    def close(self):
        if getattr(self, "h", None):
            _lib.lib().rcp_readset_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class RowTable:
    """Rows of segments.  ``seg_off`` partitions the flat segment arrays by row; inside a
    row, ``seg_group`` numbers the mask elements whose coverages are concatenated."""

    def __init__(self, seg_off, chrom, start, end, strand, seg_group=None, group_is_list=None,
                 ignore_strand=True, names=None):
        self.seg_off = np.ascontiguousarray(seg_off, dtype=np.int64)
        self.chrom = np.ascontiguousarray(chrom, dtype=np.int32)
        self.start = np.ascontiguousarray(start, dtype=np.int32)
        self.end = np.ascontiguousarray(end, dtype=np.int32)
        self.strand = np.ascontiguousarray(strand, dtype=np.int8)
        self.seg_group = None if seg_group is None else np.ascontiguousarray(seg_group, dtype=np.int8)
        self.group_is_list = None if group_is_list is None else np.ascontiguousarray(group_is_list, dtype=np.uint8)
        self.ignore_strand = bool(ignore_strand)
        self.n_rows = len(self.seg_off) - 1
        self.names = names

    @classmethod
    def from_ranges(cls, chrom, start, end, strand, **kw):
        return cls(np.arange(len(start) + 1), chrom, start, end, strand, **kw)

    def desc(self):
        return _lib.RowsDesc(self.n_rows, cptr(self.seg_off, _lib._i64p), cptr(self.chrom, _lib._i32p),
                             cptr(self.start, _lib._i32p), cptr(self.end, _lib._i32p),
                             cptr(self.strand, _lib._i8p), cptr(self.seg_group, _lib._i8p),
                             cptr(self.group_is_list, _lib._u8p), int(self.ignore_strand))


WHERE = {"whole": 0, "center": 1, "upstream": 2, "downstream": 3}


class Bins:
    """Column parts of the profile row (R/profile.R slices) and the splitVector options.

    ``parts`` is a list of ``(where, n_bins)`` or ``(where, 0, per_base_width)``; ``where`` is
    one of whole / center / upstream / downstream (binCoverageMatrix's ``where``)."""

    def __init__(self, parts, flank=(0, 0), stat="mean", interp="auto", rng_kind="Rejection", scale=1.0):
        self.parts = [tuple(p) for p in parts]
        self.where = np.array([WHERE[p[0]] if isinstance(p[0], str) else int(p[0]) for p in self.parts],
                              dtype=np.int32)
        self.n_bins = np.array([p[1] for p in self.parts], dtype=np.int32)
        self.width = np.array([p[2] if len(p) > 2 else 0 for p in self.parts], dtype=np.int32)
        self.flank = (int(flank[0]), int(flank[1]))
        self.stat = STAT[stat] if isinstance(stat, str) else int(stat)
        self.interp = INTERP[interp] if isinstance(interp, str) else int(interp)
        self.rng_kind = RNG[rng_kind] if isinstance(rng_kind, str) else int(rng_kind)
        self.scale = float(scale)

    @property
    def n_cols(self):
        return int(sum(w if b == 0 else b for b, w in zip(self.n_bins, self.width)))

    def desc(self):
        fl = (ctypes.c_int32 * 2)(*self.flank)
        return _lib.BinsDesc(len(self.parts), cptr(self.where, _lib._i32p), fl, cptr(self.n_bins, _lib._i32p),
                             cptr(self.width, _lib._i32p), self.stat, self.interp, self.rng_kind, self.scale)


class Plan:
    """One fused coverage -> profile pass of ``rows`` over ``readset`` with ``bins``."""

    def __init__(self, readset, rows, bins, kernel="auto", heavy_threshold=-1, out_ld=0, min_col_chunks=0,
                 concurrent=0):
        """``kernel``: "auto" | "general" | "lean" | "lean_any" | "rows" (rcp_plan_opts.pileup_kernel; every choice
        gives bit-identical results); ``heavy_threshold``: -1 default, 0 off; ``out_ld``: the
        output's column stride, 0 = n_rows, "padded" = the next multiple of 16 (whole 128-B
        lines per 16-row column segment), or any value >= n_rows; ``concurrent``: plans the caller
        keeps in flight on other streams (rcp_plan_opts.concurrent: > 1 leaves 1/8 of the CUs'
        workgroup slots to their locate / heavy launches)."""
        self.readset = readset  # keeps the device reads alive
        self.rows = rows
        self.bins = bins
        rd = rows.desc()
        bd = ctypes.byref(bins.desc()) if bins is not None else None
        ld = -1 if out_ld == "padded" else int(out_ld)
        opts = _lib.PlanOpts(KERNEL[kernel] if isinstance(kernel, str) else int(kernel), int(heavy_threshold), ld,
                             int(min_col_chunks), int(concurrent))
        h = ctypes.c_void_p()
        with torch.cuda.device(readset.device):
            check(_lib.lib().rcp_plan_create_ex(readset.h, ctypes.byref(rd), bd, ctypes.byref(opts),
                                                ctypes.byref(h)))
        self.h = h
        info = _lib.PlanInfo()
        check(_lib.lib().rcp_plan_info_get(self.h, ctypes.byref(info)))
        self.info = {k: getattr(info, k) for k, _ in _lib.PlanInfo._fields_}
        self.n_rows = rows.n_rows
        self.n_cols = int(info.n_cols)
        self.out_ld = int(info.out_ld)
        self.device = readset.device

    def row_lengths(self):
        out = np.zeros(self.n_rows, dtype=np.int64)
        check(_lib.lib().rcp_plan_row_lengths(self.h, cptr(out, _lib._i64p)))
        return out

    def empty_output(self):
        """The device output: (n_cols, out_ld) float64; columns [:, :n_rows] are the R matrix."""
        return torch.empty((self.n_cols, self.out_ld), dtype=torch.float64, device=f"cuda:{self.device}")

    def _check_buffers(self, out, valid, binsum):
        """The kernels write column c at out + c * out_ld: out (float64) and binsum (int64) must be
        contiguous tensors on the plan's device holding out_ld * (n_cols - 1) + n_rows elements
        (empty_output() gives (n_cols, out_ld)); valid (uint8) n_rows."""
        need = self.out_ld * (self.n_cols - 1) + self.n_rows if self.n_cols else 0
        for name, t, dt, n in (("out", out, torch.float64, need), ("binsum", binsum, torch.int64, need),
                               ("valid", valid, torch.uint8, self.n_rows)):
            if t is None:
                continue
            if not isinstance(t, torch.Tensor) or t.device != torch.device("cuda", self.device):
                raise ValueError(f"{name} must be a tensor on cuda:{self.device}")
            if t.dtype != dt or not t.is_contiguous():
                raise ValueError(f"{name} must be a contiguous {dt} tensor")
            if t.numel() < n:
                raise ValueError(f"{name} holds {t.numel()} elements; the plan writes {n} "
                                 f"(out_ld {self.out_ld} x {self.n_cols} columns)")

    def execute(self, out=None, valid=None, binsum=None, stream=None):
        """Enqueue the pass.  ``out`` is a CUDA float64 tensor holding the R column-major
        matrix with column stride ``out_ld``: shape (n_cols, out_ld) in torch's row-major terms
        (``empty_output()``), the R matrix being ``out[:, :n_rows]``.  No host sync."""
        if out is None:
            out = self.empty_output()
        self._check_buffers(out, valid, binsum)
        check(_lib.lib().rcp_plan_execute(self.h, ptr(out), ptr(valid), ptr(binsum), _stream(self.device, stream)))
        return out

    def execute_stages(self, stages, out, valid=None, binsum=None, stream=None):
        """Enqueue only some launches (1 locate, 2 pileup, 4 interpolation) -- for timing."""
        self._check_buffers(out, valid, binsum)
        check(_lib.lib().rcp_plan_execute_stages(self.h, ptr(out), ptr(valid), ptr(binsum),
                                                 _stream(self.device, stream), int(stages)))
        return out

    def status(self, stream=None):
        check(_lib.lib().rcp_plan_status(self.h, _stream(self.device, stream)))

    def heavy_rows(self, stream=None):
        """Rows the last execution piled through the skewed-row (heavy slice) path."""
        n = ctypes.c_int32()
        check(_lib.lib().rcp_plan_heavy_rows(self.h, _stream(self.device, stream), ctypes.byref(n)))
        return n.value

    def validity(self, stream=None):
        v = torch.empty(max(self.n_rows, 1), dtype=torch.uint8, device=f"cuda:{self.device}")
        check(_lib.lib().rcp_plan_validity(self.h, ptr(v), _stream(self.device, stream)))
        return v[:self.n_rows].cpu().numpy().astype(bool)

    def coverage(self, stream=None, rle=False):
        """calcCoverage: list of int32 numpy vectors (None for NULL rows); with ``rle`` each
        vector comes as its Rle ``(values, lengths)`` pair, encoded on the GPU."""
        ln = self.row_lengths()
        off = np.zeros(self.n_rows + 1, dtype=np.int64)
        off[1:] = np.cumsum(ln)
        cov = torch.empty(max(int(off[-1]), 1), dtype=torch.int32, device=f"cuda:{self.device}")
        v = torch.empty(max(self.n_rows, 1), dtype=torch.uint8, device=f"cuda:{self.device}")
        check(_lib.lib().rcp_calc_coverage(self.h, cptr(off, _lib._i64p), ptr(cov), ptr(v),
                                           _stream(self.device, stream)))
        self.status(stream)
        hv = v[:self.n_rows].cpu().numpy().astype(bool)
        if rle:
            vals = torch.empty_like(cov)
            lens = torch.empty_like(cov)
            run_off = np.zeros(self.n_rows + 1, dtype=np.int64)
            nruns = ctypes.c_int64()
            check(_lib.lib().rcp_rle_encode(self.n_rows, cptr(off, _lib._i64p), ptr(cov), self.device, ptr(vals),
                                            ptr(lens), cptr(run_off, _lib._i64p), ctypes.byref(nruns),
                                            _stream(self.device, stream)))
            hv_, hl_ = vals[:nruns.value].cpu().numpy(), lens[:nruns.value].cpu().numpy()
            return [(hv_[run_off[r]:run_off[r + 1]].copy(), hl_[run_off[r]:run_off[r + 1]].copy()) if hv[r] else None
                    for r in range(self.n_rows)]
        hc = cov.cpu().numpy()
        return [hc[off[r]:off[r + 1]].copy() if hv[r] else None for r in range(self.n_rows)]

    def run(self, stream=None, binsum=False):
        """Execute, check status, and return (R x n_cols numpy matrix (F order), valid)."""
        out = self.empty_output()
        valid = torch.empty(max(self.n_rows, 1), dtype=torch.uint8, device=f"cuda:{self.device}")
        bs = torch.empty_like(out, dtype=torch.int64) if binsum else None
        self.execute(out, valid, bs, stream)
        self.status(stream)
        mat = out[:, :self.n_rows].cpu().numpy().T  # (n_rows, n_cols) view of the column-major buffer
        v = valid[:self.n_rows].cpu().numpy().astype(bool)
        if binsum:
            return mat, v, bs[:, :self.n_rows].cpu().numpy().T
        return mat, v

    def close(self):
        if getattr(self, "h", None):
            _lib.lib().rcp_plan_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def profile_host(readset, rows, bins, out, valid=None):
    """rcp_profile: the one-shot host entry point the R .Call shim binds -- plan, one pass and
    the copy of the R column-major matrix into the caller's host array ``out`` (float64,
    C-contiguous shape (n_cols, n_rows), i.e. R's column-major n_rows x n_cols matrix) and of
    the NULL mask into ``valid`` (uint8, n_rows)."""
    if out.dtype != np.float64 or not out.flags.c_contiguous or out.size != bins.n_cols * rows.n_rows:
        raise ValueError("out must be a C-contiguous float64 array of n_cols x n_rows")
    rd = rows.desc()
    bd = bins.desc()
    with torch.cuda.device(readset.device):
        check(_lib.lib().rcp_profile(readset.h, ctypes.byref(rd), ctypes.byref(bd), cptr(out, _lib._dp),
                                     None if valid is None else cptr(valid, _lib._u8p)))
    return out


def profile_multi(readsets, rows, bins):
    """rcp_profile_multi: rows cut into one contiguous block per readset (each on its own GPU),
    one host thread per GPU, every block copied straight into the R column-major host matrix.
    Returns (matrix (n_rows, n_cols) float64, validity bool, block boundaries)."""
    rd = rows.desc()
    bd = bins.desc()
    n = len(readsets)
    hs = (ctypes.c_void_p * n)(*[r.h.value for r in readsets])
    out = np.zeros((bins.n_cols, rows.n_rows), np.float64)
    valid = np.zeros(rows.n_rows, np.uint8)
    split = np.zeros(n + 1, np.int32)
    check(_lib.lib().rcp_profile_multi(hs, n, ctypes.byref(rd), ctypes.byref(bd), cptr(out, _lib._dp),
                                       cptr(valid, _lib._u8p), cptr(split, _lib._i32p)))
    return out.T, valid.astype(bool), split


class Shards:
    """rcp_shards_create: one sample's host reads split over ``devices`` for ONE row table -- the
    rows cut into one contiguous block per device (balanced by counted candidate reads), each
    device holding only the reads its block's rows can overlap (uploaded in one slice per GPU,
    redistributed device to device).  ``devices`` may repeat a device."""

    def __init__(self, chrom, start, end, strand, seqlengths, rows, devices, strand_filter=None):
        lib = _lib.lib()
        if _lib.device_count() == 0:
            raise _lib.RcpError(-6, "no GPU visible: recoup_amd runs only on the GPU")
        self.seqlengths = np.ascontiguousarray(seqlengths, dtype=np.int64)
        runs = _chrom_runs(chrom)
        wruns = _chrom_runs(end)
        keep = [None if runs else np.ascontiguousarray(chrom, dtype=np.int32),
                np.ascontiguousarray(start, dtype=np.int32),
                None if wruns else np.ascontiguousarray(end, dtype=np.int32),
                np.ascontiguousarray(strand, dtype=np.int8)]
        sf = -1 if strand_filter is None else STRAND.get(strand_filter, strand_filter)
        d = _reads_desc(int(keep[1].shape[0]), keep, runs, self.seqlengths, 0, 0, int(sf), wruns)
        self.devices = np.ascontiguousarray(devices, dtype=np.int32)
        self.rows = rows
        rd = rows.desc()
        h = ctypes.c_void_p()
        check(lib.rcp_shards_create(ctypes.byref(d), ctypes.byref(rd), cptr(self.devices, _lib._i32p),
                                    len(self.devices), ctypes.byref(h)))
        self.h = h

    def info(self):
        """(row block boundaries [n_devices + 1] as positions of order(), reads held per device
        [n_devices])."""
        n = len(self.devices)
        split = np.zeros(n + 1, np.int32)
        reads = np.zeros(n, np.int64)
        check(_lib.lib().rcp_shards_info(self.h, None, None, cptr(split, _lib._i32p), cptr(reads, _lib._i64p)))
        return split, reads

    def order(self):
        """rcp_shards_rows: the table's row at each position of the blocks' (chromosome, start)
        order."""
        out = np.zeros(self.rows.n_rows, np.int32)
        check(_lib.lib().rcp_shards_rows(self.h, cptr(out, _lib._i32p)))
        return out

    def profile(self, bins):
        """rcp_shards_profile -> (matrix (n_rows, n_cols) float64 view of R's column-major
        matrix, validity bool)."""
        R = self.rows.n_rows
        out = np.zeros((bins.n_cols, R), np.float64)
        valid = np.zeros(max(R, 1), np.uint8)
        bd = bins.desc()
        check(_lib.lib().rcp_shards_profile(self.h, ctypes.byref(bd), cptr(out, _lib._dp), cptr(valid, _lib._u8p)))
        return out.T, valid[:R].astype(bool)

    def coverage_rle(self):
        """rcp_shards_coverage + rcp_cov_copy: (run_off, values, lengths, valid) as coverage_rle_host."""
        h = ctypes.c_void_p()
        check(_lib.lib().rcp_shards_coverage(self.h, ctypes.byref(h)))
        return _cov_copy(h)

    def coverage_rle_kept(self):
        """rcp_shards_coverage, the result kept on the devices (CoverageHandle)."""
        h = ctypes.c_void_p()
        check(_lib.lib().rcp_shards_coverage(self.h, ctypes.byref(h)))
        return CoverageHandle(h, self.rows.n_rows)

    def close(self):
        if getattr(self, "h", None):
            _lib.lib().rcp_shards_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def profile_reads(samples, seqlengths, rows, bins, device=0, outs=None, strand_filter=None):
    """rcp_profile_reads: several samples' host reads (each a tuple chrom, start, end, strand as
    ReadSet takes them) over one region table; coordinate-sorted samples given as runs stream
    through the GPU in row blocks, and sample k + 1 is uploaded while sample k is profiled and
    copied down.  ``outs``: optional caller-owned (n_cols, n_rows) float64 arrays.
    Returns [(matrix (n_rows, n_cols), validity bool)]."""
    seql = np.ascontiguousarray(seqlengths, dtype=np.int64)
    sf = -1 if strand_filter is None else STRAND.get(strand_filter, strand_filter)
    descs = []
    for chrom, start, end, strand in samples:
        runs, wruns = _chrom_runs(chrom), _chrom_runs(end)
        keep = [None if runs else np.ascontiguousarray(chrom, dtype=np.int32), np.ascontiguousarray(start, dtype=np.int32),
                None if wruns else np.ascontiguousarray(end, dtype=np.int32), np.ascontiguousarray(strand, dtype=np.int8)]
        descs.append(_reads_desc(int(keep[1].shape[0]), keep, runs, seql, int(device), 0, int(sf), wruns))
    n = len(descs)
    arr = (_lib.ReadsDesc * n)(*descs)
    if outs is None:
        outs = [np.zeros((bins.n_cols, rows.n_rows), np.float64) for _ in range(n)]
    valids = [np.zeros(max(rows.n_rows, 1), np.uint8) for _ in range(n)]
    po = (_lib._dp * n)(*[cptr(o, _lib._dp) for o in outs])
    pv = (_lib._u8p * n)(*[cptr(v, _lib._u8p) for v in valids])
    rd, bd = rows.desc(), bins.desc()
    with torch.cuda.device(int(device)):
        check(_lib.lib().rcp_profile_reads(arr, n, ctypes.byref(rd), ctypes.byref(bd), po, pv))
    return [(o.T, v[:rows.n_rows].astype(bool)) for o, v in zip(outs, valids)]


def profile_samples(readsets, rows, bins, inflight=0):
    """rcp_profile_samples: one region table over several samples' readsets (one GPU), passes
    kept ``inflight`` deep on separate HIP streams (0 = the library's default, 2), each matrix
    copied into its own host array.  Returns [(matrix (n_rows, n_cols) float64, validity bool)]."""
    rd = rows.desc()
    bd = bins.desc()
    n = len(readsets)
    hs = (ctypes.c_void_p * n)(*[r.h.value for r in readsets])
    outs = [np.zeros((bins.n_cols, rows.n_rows), np.float64) for _ in range(n)]
    valids = [np.zeros(max(rows.n_rows, 1), np.uint8) for _ in range(n)]
    po = (_lib._dp * n)(*[cptr(o, _lib._dp) for o in outs])
    pv = (_lib._u8p * n)(*[cptr(v, _lib._u8p) for v in valids])
    with torch.cuda.device(readsets[0].device if n else 0):
        check(_lib.lib().rcp_profile_samples(hs, n, ctypes.byref(rd), ctypes.byref(bd), int(inflight), po, pv))
    return [(o.T, v[:rows.n_rows].astype(bool)) for o, v in zip(outs, valids)]


def rle_arrays(coverages):
    """Flatten a coverage list (None = R's NULL, an ``Rle``-like object with ``values`` /
    ``lengths``, or a dense vector) into the run arrays of rcp_rle_desc: (run_off int64,
    lengths int32, values int32 or float64, is_null uint8).  Dense vectors are run-length
    encoded here; the values are integer when every element is (an integer Rle), else float64
    (a numeric Rle)."""
    vals, lens, nulls, counts = [], [], [], []
    for x in coverages:
        if x is None:
            nulls.append(1)
            counts.append(0)
            continue
        nulls.append(0)
        if hasattr(x, "values") and hasattr(x, "lengths"):
            v, ln = np.asarray(x.values), np.asarray(x.lengths, dtype=np.int64)
        else:
            d = np.asarray(x)
            if d.size == 0:
                v, ln = d[:0], np.zeros(0, np.int64)
            else:
                cut = np.flatnonzero(d[1:] != d[:-1]) + 1
                starts = np.concatenate([[0], cut])
                v = d[starts]
                ln = np.diff(np.concatenate([starts, [d.size]]))
        vals.append(v)
        lens.append(ln)
        counts.append(len(ln))
    run_off = np.zeros(len(counts) + 1, dtype=np.int64)
    run_off[1:] = np.cumsum(counts)
    lengths = np.ascontiguousarray(np.concatenate(lens) if lens else np.zeros(0), dtype=np.int32)
    allv = np.concatenate(vals) if vals else np.zeros(0, np.int32)
    integer = allv.dtype.kind in "iub" or (allv.dtype.kind == "f" and allv.size and
                                           np.all(np.isfinite(allv)) and np.all(allv == np.round(allv)) and
                                           np.all(np.abs(allv) < 2 ** 31))
    values = np.ascontiguousarray(allv, dtype=np.int32 if integer else np.float64)
    return run_off, lengths, values, np.asarray(nulls, dtype=np.uint8)


def profile_rle(coverages, bins, device=0):
    """rcp_profile_rle: binCoverageMatrix / baseCoverageMatrix of a host coverage list (the
    reference's list of Rle).  Returns (R x n_cols float64 matrix in R column-major (F) order,
    valid bool)."""
    return profile_rle_arrays(*rle_arrays(coverages), bins, device)


def profile_rle_arrays(run_off, lengths, values, nulls, bins, device=0, out=None):
    """rcp_profile_rle on run arrays as the R shim passes them (``.rcpRleArrays``: run_off int64
    [R + 1], lengths int32, values int32 (integer Rle) or float64 (numeric Rle), is_null uint8
    [R]).  ``out``: optional caller-owned (R, n_cols) float64 F-order matrix (R's allocMatrix)."""
    R = len(nulls)
    integer = values.dtype == np.int32
    d = _lib.RleDesc(R, cptr(run_off, _lib._i64p), cptr(lengths, _lib._i32p),
                     cptr(values, _lib._i32p) if integer else None,
                     None if integer else cptr(values, _lib._dp), cptr(nulls, _lib._u8p))
    if out is None:
        out = np.zeros((R, bins.n_cols), order="F")
    elif out.dtype != np.float64 or not out.flags.f_contiguous or out.shape != (R, bins.n_cols):
        raise ValueError("out must be an F-ordered float64 array of n_rows x n_cols")
    valid = np.zeros(max(R, 1), np.uint8)
    bd = bins.desc()
    if np.ndim(device) == 0:
        with torch.cuda.device(int(device)):
            check(_lib.lib().rcp_profile_rle(ctypes.byref(d), ctypes.byref(bd), int(device), cptr(out, _lib._dp),
                                             cptr(valid, _lib._u8p)))
    else:  # several GPUs: rcp_profile_rle_multi
        devs = np.ascontiguousarray(device, dtype=np.int32)
        check(_lib.lib().rcp_profile_rle_multi(ctypes.byref(d), ctypes.byref(bd), cptr(devs, _lib._i32p), len(devs),
                                               cptr(out, _lib._dp), cptr(valid, _lib._u8p)))
    return out, valid[:R].astype(bool)


def coverage_rle_host(readset, rows, timing=None):
    """rcp_coverage_rle + rcp_cov_copy (what the R shim's rcp_R_coverage does for calcCoverage):
    the named list of Rle as host run arrays -- (run_off int64 [R + 1], values int32, lengths
    int32, valid uint8 [R]); a row with valid 0 is the reference's NULL."""
    import time
    L = _lib.lib()
    rd = rows.desc()
    h = ctypes.c_void_p()
    t0 = time.perf_counter()
    with torch.cuda.device(readset.device):
        check(L.rcp_coverage_rle(readset.h, ctypes.byref(rd), ctypes.byref(h)))
    t1 = time.perf_counter()
    res = _cov_copy(h)
    if timing is not None:
        timing["coverage_ms"] = round((t1 - t0) * 1e3, 2)
        timing["copy_ms"] = round((time.perf_counter() - t1) * 1e3, 2)
    return res


def _cov_arrays(h):
    """rcp_cov_info + rcp_cov_copy of a coverage handle: (run_off, values, lengths, valid)."""
    L = _lib.lib()
    nr, nruns = ctypes.c_int32(), ctypes.c_int64()
    check(L.rcp_cov_info(h, ctypes.byref(nr), ctypes.byref(nruns)))
    run_off = np.empty(nr.value + 1, np.int64)
    values = np.empty(max(nruns.value, 1), np.int32)
    lengths = np.empty(max(nruns.value, 1), np.int32)
    valid = np.empty(max(nr.value, 1), np.uint8)
    check(L.rcp_cov_copy(h, cptr(run_off, _lib._i64p), cptr(values, _lib._i32p), cptr(lengths, _lib._i32p),
                         cptr(valid, _lib._u8p)))
    return run_off, values[:nruns.value], lengths[:nruns.value], valid[:nr.value]


def _cov_copy(h):
    """rcp_cov_info + rcp_cov_copy + rcp_cov_free of a coverage handle."""
    try:
        return _cov_arrays(h)
    finally:
        _lib.lib().rcp_cov_free(h)


class CoverageHandle:
    """A calcCoverage result kept on the device (rcp_coverage_rle / rcp_shards_coverage): its runs
    copied to the host (copy(): the arrays the R shim builds the list of Rle from) and profiled
    where they are (profile(): rcp_profile_cov -- what r/R/rcp.R does while the list it returned
    is unchanged, instead of uploading the runs again)."""

    def __init__(self, h, n_rows):
        self.h, self.n_rows = h, n_rows

    def copy(self):
        return _cov_arrays(self.h)

    def profile(self, bins, out=None):
        """rcp_profile_cov -> (matrix (n_rows, n_cols) F-ordered float64, validity bool)."""
        R = self.n_rows
        if out is None:
            out = np.zeros((R, bins.n_cols), order="F")
        elif out.dtype != np.float64 or not out.flags.f_contiguous or out.shape != (R, bins.n_cols):
            raise ValueError("out must be an F-ordered float64 array of n_rows x n_cols")
        valid = np.zeros(max(R, 1), np.uint8)
        bd = bins.desc()
        check(_lib.lib().rcp_profile_cov(self.h, ctypes.byref(bd), cptr(out, _lib._dp), cptr(valid, _lib._u8p)))
        return out, valid[:R].astype(bool)

    def close(self):
        if getattr(self, "h", None):
            _lib.lib().rcp_cov_free(self.h)
            self.h = None

    def __del__(self):
        self.close()


def coverage_rle_kept(readset, rows):
    """rcp_coverage_rle, the result kept on the device (CoverageHandle)."""
    rd = rows.desc()
    h = ctypes.c_void_p()
    with torch.cuda.device(readset.device):
        check(_lib.lib().rcp_coverage_rle(readset.h, ctypes.byref(rd), ctypes.byref(h)))
    return CoverageHandle(h, rows.n_rows)
