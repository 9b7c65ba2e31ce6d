"""The R side of the drop-in boundary (r/src/recoup_amd_shim.c, r/R/rcp.R), without R: the
.Call shim compiles against include/recoup_amd.h (with tests/rstub, minimal declarations of the
R C API it uses), every routine the R wrappers .Call is registered with the shim, and every
library function the shim calls is part of the header the library exports."""
import os
import re
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHIM = os.path.join(ROOT, "r", "src", "recoup_amd_shim.c")
RSRC = os.path.join(ROOT, "r", "R", "rcp.R")


def test_shim_compiles_against_the_header():
    r = subprocess.run(["gcc", "-std=c99", "-Wall", "-Wextra", "-Werror", "-Wno-unused-parameter",
                        "-Wno-cast-function-type", "-fsyntax-only", "-I", os.path.join(ROOT, "tests", "rstub"),
                        "-I", os.path.join(ROOT, "include"), SHIM], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_registered_routines_cover_the_r_wrappers():
    shim = open(SHIM).read()
    reg = dict((n, int(k)) for n, k in re.findall(r'\{"(rcp_R_\w+)", \(DL_FUNC\)&\w+, (\d+)\}', shim))
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
