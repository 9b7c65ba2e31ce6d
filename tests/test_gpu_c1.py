"""GPU parity on the reference's own fixture (config C1, data/recoup_test_data.rda).

Expected values: tests/golden/c1_expected.npz, produced by the CPU oracle (see
tests/golden/make_fixtures.py); the oracle is itself pinned in tests/test_oracle.py.
Integer per-base depth and bin numerators must be bit-exact; means within 1e-12 relative
(north_star's bar is 1e-6)."""
import os

import numpy as np
import pytest

from tests import helpers

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden", "c1_expected.npz")
MEAN_RTOL = 1e-12


@pytest.fixture(scope="module")
def c1(gpu):
    d, S, G, E = helpers.c1()
    rsets = [helpers.readset(s) for s in S]
    gold = dict(np.load(GOLD))
    return dict(S=S, G=G, E=E, rsets=rsets, gold=gold)


def _run(rs, rows, bins, binsum=False):
    from recoup_amd.engine import Plan
    return Plan(rs, rows, bins).run(binsum=binsum)


def test_tss_per_base(c1):
    from recoup_amd.engine import Bins
    rows = helpers.tss_rows(c1["G"])
    for k, rs in enumerate(c1["rsets"]):
        mat, valid = _run(rs, rows, Bins([("whole", 0, 4000)]))
        np.testing.assert_array_equal(valid, c1["gold"][f"tss_valid_s{k}"].astype(bool))
        np.testing.assert_array_equal(mat, c1["gold"][f"tss_base_s{k}"].astype(np.float64))


def test_tss_heatmap_200(c1):
    from recoup_amd.engine import Bins
    rows = helpers.tss_rows(c1["G"])
    for k, rs in enumerate(c1["rsets"]):
        mat, valid, bs = _run(rs, rows, Bins([("whole", 200)]), binsum=True)
        np.testing.assert_allclose(mat, c1["gold"][f"tss_heat_s{k}"], rtol=MEAN_RTOL, atol=0)
        np.testing.assert_array_equal(bs, np.rint(c1["gold"][f"tss_heat_s{k}"] * 20).astype(np.int64))


def test_tss_150_rng_layout(c1):
    from recoup_amd.engine import Bins
    rows = helpers.tss_rows(c1["G"])
    for k, rs in enumerate(c1["rsets"]):
        mat, _ = _run(rs, rows, Bins([("whole", 150)]))
        np.testing.assert_allclose(mat, c1["gold"][f"tss150_s{k}"], rtol=MEAN_RTOL, atol=0)


@pytest.mark.parametrize("stat", ["mean", "median"])
def test_genebody(c1, stat):
    rows = helpers.tss_rows(c1["G"], region="genebody")
    bins = helpers.unequal_bins((2000, 2000), 50, 150, stat=stat)
    for k, rs in enumerate(c1["rsets"]):
        mat, valid = _run(rs, rows, bins)
        np.testing.assert_array_equal(valid, c1["gold"][f"gb_valid_s{k}"].astype(bool))
        np.testing.assert_allclose(mat, c1["gold"][f"gb_{stat}_s{k}"], rtol=1e-9, atol=1e-12)


def test_rna(c1):
    rows = helpers.rna_rows(c1["G"], c1["E"])
    bins = helpers.unequal_bins((2000, 2000), 50, 150)
    for k, rs in enumerate(c1["rsets"]):
        mat, valid = _run(rs, rows, bins)
        np.testing.assert_array_equal(valid, c1["gold"][f"rna_valid_s{k}"].astype(bool))
        np.testing.assert_allclose(mat, c1["gold"][f"rna_s{k}"], rtol=1e-9, atol=1e-12)


def test_calc_coverage_whole_genes(c1):
    from recoup_amd.engine import Bins, Plan, RowTable
    G = c1["G"]
    rows = RowTable.from_ranges(np.zeros(len(G["start"]), np.int32), G["start"], G["end"], G["strand"])
    plan = Plan(c1["rsets"][0], rows, None)
    cov = plan.coverage()
    g = c1["gold"]
    ln = np.array([len(c) if c is not None else -1 for c in cov])
    np.testing.assert_array_equal(ln, g["calc_len"])
    np.testing.assert_array_equal([int(c.sum()) if c is not None else 0 for c in cov], g["calc_sum"])
    np.testing.assert_array_equal([int((c.astype(np.int64) * (np.arange(len(c)) % 9973)).sum())
                                   if c is not None else 0 for c in cov], g["calc_wsum"])
