"""ctypes binding of ``librecoup_amd.so`` (the C ABI declared in ``include/recoup_amd.h``).

The library is built in-tree by ``recoup_amd.build`` (hipcc, gfx950).  There is no CPU
fallback: if the library is missing or no GPU is visible, every call raises.

torch is imported before the library is loaded so that both share ONE HIP runtime
(torch ships ``libamdhip64.so.7`` with the same SONAME): device pointers and streams from
torch tensors are then valid inside the library.
"""
import ctypes
import os

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

HERE = os.path.dirname(os.path.abspath(__file__))
# RCP_LIB_PATH: an alternative build of the same library (ablation studies, tools/ablate.sh)
LIB_PATH = os.environ.get("RCP_LIB_PATH", os.path.join(HERE, "librecoup_amd.so"))

RCP_OK = 0
ERRORS = {-1: "EINVAL", -2: "EHIP", -3: "ENOMEM", -4: "EUNSUPPORTED", -5: "ESEMANTIC", -6: "ENODEVICE"}

_i32p = ctypes.POINTER(ctypes.c_int32)
_i64p = ctypes.POINTER(ctypes.c_int64)
_i8p = ctypes.POINTER(ctypes.c_int8)
_u8p = ctypes.POINTER(ctypes.c_uint8)
_dp = ctypes.POINTER(ctypes.c_double)
_vp = ctypes.c_void_p


class RcpError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"recoup_amd {ERRORS.get(code, code)}: {msg}")
        self.code = code


class SemanticError(RcpError):
    """The reference itself would raise an R error for this input."""


class UnsupportedError(RcpError):
    """Valid reference input outside what this build implements."""


class ReadsDesc(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int64), ("chrom", _vp), ("start", _vp), ("end", _vp), ("strand", _vp),
                ("n_chrom", ctypes.c_int32), ("seqlen", _i64p), ("device", ctypes.c_int32),
                ("on_device", ctypes.c_int32), ("strand_filter", ctypes.c_int32), ("n_chrom_runs", ctypes.c_int32),
                ("chrom_run_value", _i32p), ("chrom_run_length", _i64p), ("n_width_runs", ctypes.c_int32),
                ("width_run_value", _i32p), ("width_run_length", _i64p)]


class RowsDesc(ctypes.Structure):
    _fields_ = [("n_rows", ctypes.c_int32), ("seg_off", _i64p), ("seg_chrom", _i32p), ("seg_start", _i32p),
                ("seg_end", _i32p), ("seg_strand", _i8p), ("seg_group", _i8p), ("group_is_list", _u8p),
                ("ignore_strand", ctypes.c_int32)]


class BinsDesc(ctypes.Structure):
    _fields_ = [("n_parts", ctypes.c_int32), ("where", _i32p), ("flank", ctypes.c_int32 * 2), ("n_bins", _i32p),
                ("per_base_width", _i32p), ("stat", ctypes.c_int32), ("interp", ctypes.c_int32),
                ("rng_kind", ctypes.c_int32), ("scale", ctypes.c_double)]


class PlanInfo(ctypes.Structure):
    _fields_ = [("n_cols", ctypes.c_int64), ("n_segments", ctypes.c_int64), ("n_interp_rows", ctypes.c_int64),
                ("lds_bytes", ctypes.c_int64), ("grid", ctypes.c_int64), ("tile_rows", ctypes.c_int32),
                ("chunk_positions", ctypes.c_int32), ("pileup_kernel", ctypes.c_int32), ("read_bytes", ctypes.c_int32),
                ("out_ld", ctypes.c_int64), ("fold", ctypes.c_int32), ("reserved", ctypes.c_int32)]


class RleDesc(ctypes.Structure):
    _fields_ = [("n_rows", ctypes.c_int32), ("run_off", _i64p), ("lengths", _i32p), ("ivalues", _i32p),
                ("dvalues", _dp), ("is_null", _u8p)]


class PlanOpts(ctypes.Structure):
    _fields_ = [("pileup_kernel", ctypes.c_int32), ("heavy_threshold", ctypes.c_int32),
                ("out_ld", ctypes.c_int64), ("min_col_chunks", ctypes.c_int32), ("concurrent", ctypes.c_int32),
                ("reserved", ctypes.c_int32 * 2)]


# every symbol include/recoup_amd.h declares: (name, restype, argtypes)
SIGNATURES = [
    ("rcp_version", ctypes.c_char_p, []),
    ("rcp_last_error", ctypes.c_char_p, []),
    ("rcp_device_count", ctypes.c_int, [ctypes.POINTER(ctypes.c_int)]),
    ("rcp_readset_create", ctypes.c_int, [ctypes.POINTER(ReadsDesc), _vp, ctypes.POINTER(_vp)]),
    ("rcp_readset_destroy", ctypes.c_int, [_vp]),
    ("rcp_readset_info", ctypes.c_int, [_vp, _i64p, _i64p]),
    ("rcp_release_pool", ctypes.c_int, [ctypes.c_int]),
    ("rcp_plan_create", ctypes.c_int, [_vp, ctypes.POINTER(RowsDesc), ctypes.POINTER(BinsDesc), ctypes.POINTER(_vp)]),
    ("rcp_plan_create_ex", ctypes.c_int, [_vp, ctypes.POINTER(RowsDesc), ctypes.POINTER(BinsDesc),
                                          ctypes.POINTER(PlanOpts), ctypes.POINTER(_vp)]),
    ("rcp_plan_destroy", ctypes.c_int, [_vp]),
    ("rcp_plan_info_get", ctypes.c_int, [_vp, ctypes.POINTER(PlanInfo)]),
    ("rcp_plan_execute", ctypes.c_int, [_vp, _vp, _vp, _vp, _vp]),
    ("rcp_plan_execute_stages", ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, ctypes.c_int]),
    ("rcp_plan_status", ctypes.c_int, [_vp, _vp]),
    ("rcp_plan_validity", ctypes.c_int, [_vp, _vp, _vp]),
    ("rcp_plan_heavy_rows", ctypes.c_int, [_vp, _vp, _i32p]),
    ("rcp_plan_row_lengths", ctypes.c_int, [_vp, _i64p]),
    ("rcp_profile", ctypes.c_int, [_vp, ctypes.POINTER(RowsDesc), ctypes.POINTER(BinsDesc), _dp, _u8p]),
    ("rcp_readset_create_multi", ctypes.c_int, [ctypes.POINTER(ReadsDesc), _i32p, ctypes.c_int32,
                                                ctypes.POINTER(_vp)]),
    ("rcp_profile_multi", ctypes.c_int, [ctypes.POINTER(_vp), ctypes.c_int32, ctypes.POINTER(RowsDesc),
                                         ctypes.POINTER(BinsDesc), _dp, _u8p, _i32p]),
    ("rcp_shards_create", ctypes.c_int, [ctypes.POINTER(ReadsDesc), ctypes.POINTER(RowsDesc), _i32p, ctypes.c_int32,
                                         ctypes.POINTER(_vp)]),
    ("rcp_shards_info", ctypes.c_int, [_vp, _i32p, _i32p, _i32p, _i64p]),
    ("rcp_shards_rows", ctypes.c_int, [_vp, _i32p]),
    ("rcp_shards_profile", ctypes.c_int, [_vp, ctypes.POINTER(BinsDesc), _dp, _u8p]),
    ("rcp_shards_coverage", ctypes.c_int, [_vp, ctypes.POINTER(_vp)]),
    ("rcp_shards_destroy", ctypes.c_int, [_vp]),
    ("rcp_profile_rle_multi", ctypes.c_int, [ctypes.POINTER(RleDesc), ctypes.POINTER(BinsDesc), _i32p, ctypes.c_int32,
                                             _dp, _u8p]),
    ("rcp_profile_reads", ctypes.c_int, [ctypes.POINTER(ReadsDesc), ctypes.c_int32, ctypes.POINTER(RowsDesc),
                                         ctypes.POINTER(BinsDesc), ctypes.POINTER(_dp), ctypes.POINTER(_u8p)]),
    ("rcp_profile_samples", ctypes.c_int, [ctypes.POINTER(_vp), ctypes.c_int32, ctypes.POINTER(RowsDesc),
                                           ctypes.POINTER(BinsDesc), ctypes.c_int32, ctypes.POINTER(_dp),
                                           ctypes.POINTER(_u8p)]),
    ("rcp_calc_coverage", ctypes.c_int, [_vp, _i64p, _vp, _vp, _vp]),
    ("rcp_profile_rle", ctypes.c_int, [ctypes.POINTER(RleDesc), ctypes.POINTER(BinsDesc), ctypes.c_int, _dp, _u8p]),
    ("rcp_rle_encode", ctypes.c_int, [ctypes.c_int32, _i64p, _vp, ctypes.c_int, _vp, _vp, _i64p, _i64p, _vp]),
    ("rcp_coverage_rle", ctypes.c_int, [_vp, ctypes.POINTER(RowsDesc), ctypes.POINTER(_vp)]),
    ("rcp_cov_info", ctypes.c_int, [_vp, _i32p, _i64p]),
    ("rcp_cov_copy", ctypes.c_int, [_vp, _i64p, _i32p, _i32p, _u8p]),
    ("rcp_cov_free", ctypes.c_int, [_vp]),
    ("rcp_profile_cov", ctypes.c_int, [_vp, ctypes.POINTER(BinsDesc), _dp, _u8p]),
    ("rcp_bam_read", ctypes.c_int, [ctypes.c_char_p, ctypes.c_int, ctypes.c_double, ctypes.c_int,
                                    ctypes.POINTER(_vp)]),
    ("rcp_bam_info", ctypes.c_int, [_vp, _i64p, _i32p, _i64p]),
    ("rcp_bam_ref_name", ctypes.c_char_p, [_vp, ctypes.c_int32]),
    ("rcp_bam_copy", ctypes.c_int, [_vp, _i64p, _i32p, _i32p, _i32p, _i8p]),
    ("rcp_bam_free", ctypes.c_int, [_vp]),
    ("rcp_rng_create", ctypes.c_int, [ctypes.c_uint32, ctypes.c_int, ctypes.POINTER(_vp)]),
    ("rcp_rng_unif", ctypes.c_int, [_vp, ctypes.c_int64, _dp]),
    ("rcp_rng_sample_sorted", ctypes.c_int, [_vp, ctypes.c_int64, ctypes.c_int64, _i64p]),
    ("rcp_rng_free", ctypes.c_int, [_vp]),
]

_LIB = None


def lib():
    """Load the in-tree library (raises if it has not been built)."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} is missing: run `python -c 'import __graft_entry__ as g; g.build()'`"
                              " (hipcc --offload-arch=gfx950); recoup_amd has no CPU fallback")
        L = ctypes.CDLL(LIB_PATH)
        # an A/B variant library (RCP_LIB_PATH, tools/gpu_ab.sh) built from an older tree may
        # lack entry points added since; the in-tree library must export every one
        variant = "RCP_LIB_PATH" in os.environ
        for name, res, args in SIGNATURES:
            if variant and not hasattr(L, name):
                continue
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _LIB = L
    return _LIB


def check(rc):
    if rc != RCP_OK:
        msg = lib().rcp_last_error().decode(errors="replace")
        cls = {-4: UnsupportedError, -5: SemanticError}.get(rc, RcpError)
        raise cls(rc, msg)
    return rc


def device_count():
    n = ctypes.c_int(0)
    check(lib().rcp_device_count(ctypes.byref(n)))
    return n.value


def ptr(t):
    """Raw data pointer of a numpy array or torch tensor (None -> NULL)."""
    if t is None:
        return None
    if isinstance(t, torch.Tensor):
        return ctypes.c_void_p(t.data_ptr())
    return ctypes.c_void_p(t.ctypes.data)


def cptr(a, ctype):
    return None if a is None else a.ctypes.data_as(ctype)


def stream_handle(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)
