"""The strong-scaled bench's data path on CPU (what `bench.py --gpus N` does per rank before the
GPU sees anything): bench.shard_of cuts the region table into N contiguous shards balanced by
overlapping reads, bench.subset_rows takes a shard's rows and bench.reads_for_rows keeps only the
reads that shard can touch.  Every shard's profile, computed by the oracle from its own reads,
must equal its rows of the whole-table profile bit for bit (validity included), for known and NA
seqlengths and uneven N -- the property that lets the ranks share no data-path collective."""
import numpy as np
import pytest
import torch

import bench
from recoup_amd.engine import Bins, RowTable
from tests import oracle_rows

CHROM_LEN = np.array([300_000, 180_000, 60_000], dtype=np.int64)


def _workload(seed=3, n=40_000, R=240, width=2000):
    rng = np.random.default_rng(seed)
    chrom = rng.integers(0, 3, n).astype(np.int32)
    hot = rng.random(n) < 0.4
    start = np.where(hot, rng.integers(10_000, 12_000, n), rng.integers(1, 50_000, n)).astype(np.int64)
    start = np.minimum(start, CHROM_LEN[chrom] - 400)
    end = start + rng.integers(20, 300, n) - 1
    strand = rng.integers(0, 3, n).astype(np.int8)
    reads = (chrom, start.astype(np.int32), end.astype(np.int32), strand)
    rc = rng.integers(0, 3, R).astype(np.int32)
    rs = rng.integers(1, 55_000, R).astype(np.int64)
    o = np.lexsort((rs, rc))  # (chromosome, start) order, as the synthetic tables are
    rc, rs = rc[o], rs[o]
    st = rng.integers(0, 3, R).astype(np.int8)
    return reads, RowTable.from_ranges(rc, rs, rs + width - 1, st)


def _overlaps(reads, rows):
    chrom, start, end, _ = reads
    out = np.zeros(rows.n_rows, np.int64)
    for r in range(rows.n_rows):
        out[r] = int(np.count_nonzero((chrom == rows.chrom[r]) & (start <= rows.end[r]) & (end >= rows.start[r])))
    return out


@pytest.mark.parametrize("seqlen", [CHROM_LEN, np.full(3, -1, np.int64)], ids=["known", "NA"])
def test_shards_reproduce_whole_profile(seqlen):
    reads, rows = _workload()
    bins = Bins([("whole", 100)])
    full, fvalid = oracle_rows.profile(oracle_rows.row_coverage(oracle_rows.index_for(reads, seqlen), rows), bins)
    assert fvalid.sum() > 0
    ovl = _overlaps(reads, rows)
    treads = tuple(torch.as_tensor(x) for x in reads)
    for world in (2, 3, 8):
        covered = 0
        for rank in range(world):
            lo, hi, cuts = bench.shard_of(rows, ovl, world, rank)
            assert cuts[0] == 0 and cuts[-1] == rows.n_rows
            sub = bench.subset_rows(rows, lo, hi)
            assert sub.n_rows == hi - lo
            sr = tuple(t.numpy() for t in bench.reads_for_rows(treads, sub, len(CHROM_LEN)))
            assert len(sr[1]) <= len(reads[1])
            if sub.n_rows == 0:
                continue
            got, gvalid = oracle_rows.profile(oracle_rows.row_coverage(oracle_rows.index_for(sr, seqlen), sub), bins)
            np.testing.assert_array_equal(gvalid, fvalid[lo:hi])
            np.testing.assert_array_equal(got.view(np.uint64), full[lo:hi].view(np.uint64))
            covered += hi - lo
        assert covered == rows.n_rows


def test_shards_balance_by_overlaps():
    """A hot region of rows takes a shard of its own size in reads, not in rows."""
    reads, rows = _workload(seed=5)
    ovl = _overlaps(reads, rows)
    w = ovl.astype(np.float64) + 64.0
    for world in (2, 4):
        loads = []
        for rank in range(world):
            lo, hi, _ = bench.shard_of(rows, ovl, world, rank)
            loads.append(w[lo:hi].sum())
        assert max(loads) <= w.sum() / world + w.max() + 1e-9


class _Args:
    def __init__(self, gpus):
        self.gpus = gpus


def test_gpus_flag_reaches_the_world_size():
    """`bench.py --gpus N` without a launcher starts N ranks as a child torch.distributed.run
    (the driver may run it either way); under a launcher --gpus must match WORLD_SIZE."""
    argv = ["--gpus", "8", "--steps", "5"]
    world, cmd = bench.launch_plan(_Args(8), {}, 8, argv, port=29555)
    assert world == 8 and cmd is not None
    assert cmd[1:4] == ["-m", "torch.distributed.run", "--nnodes=1"]
    assert "--nproc-per-node=8" in cmd and cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-len(argv):] == argv and cmd[-len(argv) - 1].endswith("bench.py")
    # one GPU: run here; no flag under a launcher: the launcher's world
    assert bench.launch_plan(_Args(None), {}, 1, []) == (1, None)
    assert bench.launch_plan(_Args(None), {"WORLD_SIZE": "4"}, 8, []) == (4, None)
    assert bench.launch_plan(_Args(4), {"WORLD_SIZE": "4"}, 8, []) == (4, None)
    # a rehearsal: two ranks sharing one GPU
    world, cmd = bench.launch_plan(_Args(2), {"RCP_SHARE_GPU": "1"}, 1, ["--gpus", "2"])
    assert world == 2 and "--nproc-per-node=2" in cmd
    assert bench.devices_used(2, 1, True) == 1 and bench.devices_used(8, 8, False) == 8


@pytest.mark.parametrize("args,env,visible", [
    (8, {}, 1),                      # fewer GPUs than asked for
    (2, {}, 0),
    (1, {}, 0),                      # no GPU at all
    (4, {"WORLD_SIZE": "2"}, 8),     # --gpus disagrees with the launcher
    (None, {"WORLD_SIZE": "8"}, 2),  # the launcher started more ranks than GPUs
])
def test_gpus_flag_refuses_what_cannot_run(args, env, visible):
    with pytest.raises(SystemExit) as e:
        bench.launch_plan(_Args(args), env, visible, [])
    assert e.value.code == 2
