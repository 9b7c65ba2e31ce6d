import numpy as np, ctypes, sys
sys.path.insert(0, '.')
from tests import helpers
from tests.test_gpu_abi import _profile
from recoup_amd import _lib
from recoup_amd.engine import Bins, Plan
d, S, G, E = helpers.c1()
rs = helpers.readset(S[0])
rows = helpers.tss_rows(G)
print("rows", rows.n_rows)
rc, out, valid = _profile(rs, rows, Bins([("whole", 0, 4000)]))
print("rc", rc, _lib.lib().rcp_last_error())
p = Plan(rs, rows, Bins([("whole", 0, 4000)]))
print(p.info)
try:
    p.run()
except Exception as e:
    print("run failed", e)
