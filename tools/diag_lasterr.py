"""Which library call leaves a HIP error in the thread's last-error slot (a later launch's
hipGetLastError reports it): the test_gpu_abi sequence around rcp_release_pool, with
hipPeekAtLastError after each step."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from recoup_amd import _lib  # noqa: E402
from recoup_amd.engine import Bins, Plan, ReadSet  # noqa: E402
from tests.test_gpu_random import CHROM_LEN, make_reads, single_rows  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so")
hip.hipPeekAtLastError.restype = ctypes.c_int
hip.hipGetErrorString.restype = ctypes.c_char_p


def peek(tag):
    e = hip.hipPeekAtLastError()
    print(f"{tag}: last error {e} {hip.hipGetErrorString(e).decode() if e else ''}", flush=True)


def profile(rs, rows, bins):
    rd, bd = rows.desc(), bins.desc()
    out = np.full((rows.n_rows, bins.n_cols), np.nan, order="F")
    valid = np.zeros(rows.n_rows, np.uint8)
    rc = _lib.lib().rcp_profile(rs.h, ctypes.byref(rd), ctypes.byref(bd), out.ctypes.data_as(_lib._dp),
                                valid.ctypes.data_as(_lib._u8p))
    return rc, out


rng = np.random.default_rng(4099)
reads = make_reads(rng, 300_000)
peek("start")
rs = ReadSet(*reads, CHROM_LEN, device=0)
peek("readset")
rows = single_rows(rng, 4099, 4000)
bins = Bins([("whole", 4000)])
ref, rv = Plan(rs, rows, bins).run()
peek("plan run")
rc, out = profile(rs, rows, bins)
peek(f"rcp_profile rc {rc} equal {np.array_equal(out.view(np.uint64), np.asfortranarray(ref).view(np.uint64))}")
del rs
peek("readset freed")
print("release", _lib.lib().rcp_release_pool(0))
peek("release_pool")
rs = ReadSet(*reads, CHROM_LEN, device=0)
peek("readset again")
