"""Execute the R .Call shim (r/src/recoup_amd_shim.c) from Python through rmini.c, a small
emulation of the R C API (test infrastructure; R is not installed here or on the GPU box).

``Shim().call(name, *args)`` is ``.Call(name, ...)``: Python values become R objects
(``numpy`` int32 -> integer, float64 -> double, bool -> logical, ``str`` -> character,
``list`` -> list, ``None`` -> NULL, ``RChar([...])`` -> a character vector) and the result comes
back as Python values (a named R list -> ``dict``, a matrix -> ``RArray``: a 2-D ``numpy`` array in
R's column-major order whose ``dimnames`` is R's ``dimnames(m)``: None, or (rownames, colnames),
each None or a list of str).  An R error raised by
the shim becomes ``RError``; the protect stack must be balanced on return.

build() compiles the shim with rmini.c against include/recoup_amd.h and links
recoup_amd/librecoup_amd.so (in-tree, like every other native piece)."""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
OUT = os.path.join(HERE, "build", "librmini_shim.so")
SRCS = [os.path.join(HERE, "rmini.c"), os.path.join(ROOT, "r", "src", "recoup_amd_shim.c")]
LIBDIR = os.path.join(ROOT, "recoup_amd")

INTSXP, LGLSXP, REALSXP, STRSXP, VECSXP, CHARSXP, NILSXP, EXTPTRSXP = 13, 10, 14, 16, 19, 9, 0, 22


class RError(Exception):
    pass


class RChar(list):
    """An R character vector (``c("a", "b")``); a plain ``str`` is a length-1 one."""


class RArray(np.ndarray):
    """An R matrix: the values plus R's ``dimnames`` (None, or a (rownames, colnames) pair)."""

    def __new__(cls, a, dimnames=None):
        obj = np.asarray(a).view(cls)
        obj.dimnames = dimnames
        return obj

    def __array_finalize__(self, obj):
        self.dimnames = getattr(obj, "dimnames", None)

    @property
    def rownames(self):
        return None if self.dimnames is None else self.dimnames[0]

    @property
    def colnames(self):
        return None if self.dimnames is None else self.dimnames[1]


def build(force=False):
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    deps = SRCS + [os.path.join(ROOT, "include", "recoup_amd.h"), os.path.join(LIBDIR, "librecoup_amd.so")]
    if not force and os.path.exists(OUT) and all(os.path.getmtime(d) <= os.path.getmtime(OUT) for d in deps):
        return OUT
    cmd = ["gcc", "-std=c99", "-O1", "-g", "-fPIC", "-shared", "-Wall", "-Wno-unused-parameter",
           "-I", os.path.join(ROOT, "tests", "rstub"), "-I", os.path.join(ROOT, "include"), "-o", OUT] + SRCS + \
          ["-L", LIBDIR, "-lrecoup_amd", "-Wl,-rpath," + LIBDIR, "-lm"]
    subprocess.check_call(cmd)
    return OUT


_SHIM = None


class Shim:
    """The shim's registered routines, called as R would call them."""

    def __init__(self):
        from recoup_amd import _lib
        _lib.lib()  # torch first: the library shares torch's HIP runtime
        L = ctypes.CDLL(OUT)
        v = ctypes.c_void_p
        L.rmini_call.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.POINTER(v), ctypes.POINTER(v),
                                 ctypes.POINTER(ctypes.c_int)]
        L.rmini_error.restype = ctypes.c_char_p
        L.rmini_routine.restype = v
        L.rmini_routine.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_int)]
        L.rmini_vector.restype = v
        L.rmini_vector.argtypes = [ctypes.c_int, ctypes.c_ssize_t, v]
        L.rmini_string.restype = v
        L.rmini_string.argtypes = [ctypes.c_char_p]
        L.rmini_list.restype = v
        L.rmini_list.argtypes = [ctypes.c_int, ctypes.POINTER(v)]
        for f in ("rmini_type", "rmini_dim"):
            getattr(L, f).argtypes = [v] + ([ctypes.c_int] if f == "rmini_dim" else [])
        L.rmini_length.restype = ctypes.c_ssize_t
        L.rmini_length.argtypes = [v]
        L.rmini_data.restype = v
        L.rmini_data.argtypes = [v]
        L.rmini_names.restype = v
        L.rmini_names.argtypes = [v]
        L.rmini_dimnames.restype = v
        L.rmini_dimnames.argtypes = [v]
        L.rmini_strings.restype = v
        L.rmini_strings.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_char_p)]
        L.rmini_nil.restype = v
        L.rmini_s4.restype = v
        L.rmini_s4.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(v)]
        L.rmini_fail_alloc_after.argtypes = [ctypes.c_long]
        assert L.rmini_init() == 0, "R_init_recoup registered no routines"
        self.L = L
        self._keep = []

    # ------------------------------------------------------------------ conversion
    def to_r(self, x):
        L = self.L
        if x is None:
            return L.rmini_nil()
        if isinstance(x, RObj):
            return x.ptr
        if isinstance(x, RChar):
            enc = [str(e).encode() for e in x]
            arr = (ctypes.c_char_p * max(len(enc), 1))(*enc)
            return L.rmini_strings(len(enc), arr)
        if isinstance(x, str):
            return L.rmini_string(x.encode())
        if isinstance(x, (list, tuple)):
            elts = (ctypes.c_void_p * max(len(x), 1))(*[self.to_r(e) for e in x])
            return L.rmini_list(len(x), elts)
        a = np.asarray(x)
        if a.dtype == np.bool_:
            a, t = a.astype(np.int32), LGLSXP
        elif np.issubdtype(a.dtype, np.integer):
            a, t = a.astype(np.int32), INTSXP
        else:
            a, t = a.astype(np.float64), REALSXP
        a = np.ascontiguousarray(a.ravel(order="F"))
        return L.rmini_vector(t, a.size, a.ctypes.data if a.size else None)

    def s4(self, **slots):
        """An S4 object with these slots (e.g. an S4Vectors::Rle: values, lengths), made once: the
        RObj passes the SAME R object to every later call (R's object identity)."""
        names = [k.encode() for k in slots]
        arr = (ctypes.c_char_p * max(len(names), 1))(*names)
        vals = (ctypes.c_void_p * max(len(names), 1))(*[self.to_r(x) for x in slots.values()])
        return RObj(self.L.rmini_s4(len(names), arr, vals))

    def from_r(self, p):
        L = self.L
        t = L.rmini_type(p)
        n = L.rmini_length(p)
        if t == NILSXP:
            return None
        if t == EXTPTRSXP:
            return RObj(p)
        if t in (INTSXP, LGLSXP, REALSXP):
            ct = ctypes.c_double if t == REALSXP else ctypes.c_int32
            a = np.ctypeslib.as_array((ct * max(n, 1)).from_address(L.rmini_data(p)))[:n].copy()
            if t == LGLSXP:
                a = a.astype(bool)
            nr, nc = L.rmini_dim(p, 0), L.rmini_dim(p, 1)
            if nr or nc:
                dn = L.rmini_dimnames(p)
                dn = None if L.rmini_type(dn) == NILSXP else tuple(self.from_r(dn))
                return RArray(a.reshape((nr, nc), order="F"), dn)
            return a
        if t == CHARSXP:
            return ctypes.string_at(L.rmini_data(p), n).decode()
        if t in (STRSXP, VECSXP):
            elts = (ctypes.c_void_p * max(n, 1)).from_address(L.rmini_data(p))
            vals = [self.from_r(elts[i]) if elts[i] else None for i in range(n)]
            nm = L.rmini_names(p)
            if L.rmini_type(nm) == STRSXP:
                return dict(zip(self.from_r(nm), vals))
            return vals
        raise TypeError(f"R type {t}")

    # ------------------------------------------------------------------ .Call
    def call(self, name, *args, raw=False):
        a = (ctypes.c_void_p * max(len(args), 1))(*[self.to_r(x) for x in args])
        out = ctypes.c_void_p()
        depth = ctypes.c_int()
        rc = self.L.rmini_call(name.encode(), len(args), a, ctypes.byref(out), ctypes.byref(depth))
        if rc == 2:
            raise TypeError(self.L.rmini_error().decode())
        if rc == 1:
            raise RError(self.L.rmini_error().decode())
        assert depth.value == 0, f"{name} returned with {depth.value} objects left on the protect stack"
        return RObj(out.value) if raw else self.from_r(out.value)

    def routine_arity(self, name):
        k = ctypes.c_int()
        self.L.rmini_routine(name.encode(), ctypes.byref(k))
        return k.value

    def fail_alloc_after(self, k):
        self.L.rmini_fail_alloc_after(int(k))

    def run_finalizers(self):
        return self.L.rmini_run_finalizers()

    def live_handles(self):
        return self.L.rmini_live_handles()

    def unguarded_handles(self):
        return self.L.rmini_unguarded_handles()


class RObj:
    """An R object passed back in as is (an external pointer: a readset)."""

    def __init__(self, ptr):
        self.ptr = ptr


def shim():
    global _SHIM
    if _SHIM is None:
        if not os.path.exists(OUT):
            raise RuntimeError(f"{OUT} is not built (python -c 'import __graft_entry__ as g; g.build()')")
        _SHIM = Shim()
    return _SHIM
