"""The C-ABI drop-in boundary (include/recoup_amd.h) without a GPU: the in-tree library loads,
exports exactly the declared entry points with default visibility, and every entry point that
needs a device fails loudly (RCP_ENODEVICE / RcpError) instead of computing on the CPU."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest
import torch

from recoup_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "recoup_amd.h")


def header_symbols():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"RCP_API\s+[\w\s\*]+?\b(rcp_\w+)\s*\(", txt)))


def test_header_declares_the_boundary():
    syms = header_symbols()
    for s in ("rcp_readset_create", "rcp_plan_create", "rcp_plan_execute", "rcp_profile", "rcp_calc_coverage"):
        assert s in syms
    assert sorted(n for n, _, _ in _lib.SIGNATURES) == syms  # the ctypes table covers the header


def test_library_loads_and_exports_every_symbol():
    L = _lib.lib()
    for s in header_symbols():
        assert hasattr(L, s), s
    nm = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True, check=True)
    exported = {ln.split()[-1] for ln in nm.stdout.splitlines() if " T " in ln}
    rcp = {s for s in exported if s.startswith("rcp_")}
    # rcp_launch_* / rcp_sort_* are internal (hidden visibility)
    assert rcp == set(header_symbols()), rcp ^ set(header_symbols())


def test_library_is_gfx950_code():
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-n", _lib.LIB_PATH], capture_output=True,
                         text=True)
    bundles = subprocess.run(["/opt/rocm/lib/llvm/bin/clang-offload-bundler", "--list", "--type=o",
                              f"--input={_lib.LIB_PATH}"], capture_output=True, text=True)
    txt = out.stdout + bundles.stdout + open(_lib.LIB_PATH, "rb").read().decode("latin1")
    assert "gfx950" in txt


def test_version_and_errors():
    L = _lib.lib()
    assert L.rcp_version().decode().startswith("recoup_amd")
    n = ctypes.c_int(-1)
    assert L.rcp_device_count(ctypes.byref(n)) == 0
    assert L.rcp_device_count(None) == -1  # RCP_EINVAL
    assert b"NULL" in L.rcp_last_error()


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-device behaviour")
def test_no_device_fails_loudly():
    L = _lib.lib()
    assert _lib.device_count() == 0
    s = np.array([1, 5], np.int32)
    e = np.array([10, 20], np.int32)
    c = np.zeros(2, np.int32)
    st = np.zeros(2, np.int8)
    sl = np.array([100], np.int64)
    d = _lib.ReadsDesc(2, _lib.ptr(c), _lib.ptr(s), _lib.ptr(e), _lib.ptr(st), 1, _lib.cptr(sl, _lib._i64p), 0, 0, -1)
    h = ctypes.c_void_p()
    assert L.rcp_readset_create(ctypes.byref(d), None, ctypes.byref(h)) == -6  # RCP_ENODEVICE
    assert not h.value
    dev = np.zeros(2, np.int32)
    hs = (ctypes.c_void_p * 2)()
    assert L.rcp_readset_create_multi(ctypes.byref(d), _lib.cptr(dev, _lib._i32p), 2, hs) == -6
    assert not hs[0] and not hs[1]
    with pytest.raises(_lib.RcpError):
        from recoup_amd.engine import ReadSet
        ReadSet(c, s, e, st, sl)
    # the high-level API refuses too (no silent CPU path)
    import recoup_amd as ra
    gr = ra.GRanges(["chr1"] * 2, s, e, ["+", "+"], seqlengths={"chr1": 100})
    with pytest.raises(_lib.RcpError):
        ra.calcCoverage(gr, gr)


def test_null_arguments_are_rejected():
    L = _lib.lib()
    assert L.rcp_readset_create(None, None, None) == -1
    assert L.rcp_plan_create(None, None, None, None) == -1
    assert L.rcp_profile_multi(None, 1, None, None, None, None, None) == -1
    assert L.rcp_readset_create_multi(None, None, 1, None) == -1
    assert L.rcp_plan_destroy(None) == 0 or L.rcp_plan_destroy(None) == -1


# header struct -> ctypes mirror in recoup_amd/_lib.py
STRUCTS = {"rcp_reads_desc": "ReadsDesc", "rcp_rows_desc": "RowsDesc", "rcp_bins_desc": "BinsDesc",
           "rcp_plan_info": "PlanInfo", "rcp_plan_opts": "PlanOpts", "rcp_rle_desc": "RleDesc"}


def test_struct_layouts_match_the_header(tmp_path):
    """Every descriptor struct the ctypes binding passes has the header's size and field offsets
    (a C probe compiled with gcc against include/recoup_amd.h prints them)."""
    lines = ["#include <stdio.h>", "#include <stddef.h>", '#include "recoup_amd.h"', "int main(void) {"]
    for c, py in STRUCTS.items():
        lines.append(f'  printf("{c} size %zu\\n", sizeof({c}));')
        for name, _ in getattr(_lib, py)._fields_:
            lines.append(f'  printf("{c} {name} %zu\\n", offsetof({c}, {name}));')
    lines += ["  return 0;", "}"]
    src = tmp_path / "probe.c"
    src.write_text("\n".join(lines) + "\n")
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    got = {}
    for ln in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.splitlines():
        c, f, v = ln.split()
        got[(c, f)] = int(v)
    for c, py in STRUCTS.items():
        cls = getattr(_lib, py)
        assert ctypes.sizeof(cls) == got[(c, "size")], c
        for name, _ in cls._fields_:
            assert getattr(cls, name).offset == got[(c, name)], (c, name)
