"""Small general-kernel tables run as row blocks (rcp_plan_opts.row_split = 0, the default): three
plans of whole 16-row tiles on their own streams, forked from the caller's stream and joined back.
Every result must be the bits of the same table run as one plan (row_split = 1): means, numerators,
validity, heavy rows, medians and interpolated rows, strand-split layouts, stage-by-stage
execution and a calcCoverage pass on the same plan."""
import numpy as np
import pytest
import torch

from tests.test_gpu_random import CHROM_LEN, make_reads, single_rows

pytestmark = pytest.mark.gpu


def run(plan, stages=None):
    out = plan.empty_output()
    valid = torch.zeros(plan.n_rows, dtype=torch.uint8, device=out.device)
    binsum = torch.zeros_like(out, dtype=torch.int64)
    if stages:
        for st in stages:
            plan.execute_stages(st, out, valid, binsum)
    else:
        plan.execute(out, valid, binsum)
    plan.status()
    torch.cuda.synchronize()
    return (out[:, :plan.n_rows].cpu().numpy(), valid.cpu().numpy(), binsum[:, :plan.n_rows].cpu().numpy(),
            plan.heavy_rows())


def same(a, b):
    for x, y in zip(a[:3], b[:3]):
        assert np.array_equal(np.ascontiguousarray(x).view(np.uint64), np.ascontiguousarray(y).view(np.uint64))
    assert a[3] == b[3]


@pytest.mark.parametrize("ignore_strand", [True, False])
def test_split_plans_bit_equal(gpu, ignore_strand):
    from recoup_amd.engine import Bins, Plan, ReadSet, RowTable
    rng = np.random.default_rng(31 + ignore_strand)
    chrom, start, end, strand = make_reads(rng, 400_000, widths=(150, 150))
    hot = rng.integers(0, 400_000, 60_000)  # a hot peak: heavy rows in one block
    chrom[hot], start[hot] = 0, 200_000 + rng.integers(0, 200, hot.size).astype(np.int32)
    end[hot] = start[hot] + 149
    rs = ReadSet(chrom, start, end, strand, CHROM_LEN, device=0)
    r0 = single_rows(rng, 9000, 2000, edge=True)
    r0.start[1], r0.end[1] = 1, 2000
    r0.chrom[5:9], r0.start[5:9] = 0, 199_500
    r0.end[5:9] = r0.start[5:9] + 1999
    rows = RowTable(r0.seg_off, r0.chrom, r0.start, r0.end, r0.strand, ignore_strand=ignore_strand)
    for bins in (Bins([("whole", 1000)]), Bins([("whole", 200)], stat="median"), Bins([("whole", 3000)])):
        split = Plan(rs, rows, bins, out_ld="padded")
        one = Plan(rs, rows, bins, out_ld="padded", row_split=1)
        assert split.info["pileup_kernel"] == 0  # the general kernel: split by default
        a = run(split)
        b = run(one)
        same(a, b)
        assert a[3] > 0  # the hot peak's rows took the heavy path
        same(run(split, stages=(1, 2, 4)), b)
        same(run(split), b)  # again (the blocks' status sets alternate)
        np.testing.assert_array_equal(split.validity(), one.validity())
    cov_split = Plan(rs, rows, Bins([("whole", 1000)])).coverage()
    cov_one = Plan(rs, rows, Bins([("whole", 1000)]), row_split=1).coverage()
    for x, y in zip(cov_split, cov_one):
        assert (x is None and y is None) or np.array_equal(x, y)


def test_split_only_small_general_tables(gpu):
    """Tables outside 4096..65536 rows, forced kernels and plans with samples in flight stay one
    plan (nothing to compare but the bits)."""
    from recoup_amd.engine import Bins, Plan, ReadSet
    rng = np.random.default_rng(5)
    rs = ReadSet(*make_reads(rng, 50_000), CHROM_LEN, device=0)
    bins = Bins([("whole", 1000)])
    small = single_rows(rng, 1000, 2000)
    a = run(Plan(rs, small, bins))
    b = run(Plan(rs, small, bins, kernel="general"))
    same(a, b)
    rows = single_rows(rng, 5000, 2000)
    c = run(Plan(rs, rows, bins, concurrent=2))
    d = run(Plan(rs, rows, bins, row_split=1))
    same(c, d)
