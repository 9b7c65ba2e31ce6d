"""Region sharding (recoup_amd/shard.py) with world_size 2 over gloo on CPU.

The per-rank compute is the oracle here (CPU test infrastructure); on GPU ranks the same
function runs the HIP engine (shard.gpu_compute).  The reassembled matrix must equal the
single-process result bit for bit, whatever the balance of the shards."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import recoup_amd as ra
from recoup_amd import shard


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _case(seed=0):
    rng = np.random.default_rng(seed)
    levels = ["chr1", "chr2", "chr3"]
    L = np.array([60000, 40000, 30000])
    n = 20000
    c = rng.integers(0, 3, n)
    hot = rng.random(n) < 0.5  # skew: half the reads pile on chr1:10k-12k
    st = np.where(hot & (c == 0), rng.integers(10000, 12000, n), rng.integers(1, L[c] - 200, n))
    reads = ra.GRanges(np.array(levels)[c], st, width=180, strand=rng.integers(0, 3, n),
                       seqlevels=levels, seqlengths=dict(zip(levels, L.tolist())))
    R = 300
    rc = rng.integers(0, 4, R)  # code 3 = chrUn (not in the reads: NULL rows)
    names = np.array(levels + ["chrUn"])[rc]
    summit = rng.integers(1, 30000, R)
    regions = ra.getRegionalRanges(ra.GRanges(names, summit, summit, rng.integers(0, 2, R),
                                              seqlevels=levels + ["chrUn"]), "custom", (500, 500))
    return reads, regions


def _oracle_compute(n_bins):
    from oracle import oracle as o

    def run(reads, regions):
        codes = regions.codes_in(reads.seqlevels)
        ix = o.Index(reads.seqcodes, reads.start, reads.end, reads.strand, reads.seqlengths)
        mask = o.Mask.from_ranges(codes, regions.start, regions.end, regions.strand)
        m, v = o.profile_part(ix, mask, n_bins)
        return m, v.astype(bool)
    return run


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        reads, regions = _case()
        out, v = shard.profile_sharded(reads, regions, _oracle_compute(50))
        mine, m, _ = shard.profile_sharded(reads, regions, _oracle_compute(50), gather=None)
        q.put((rank, out, v, len(mine)))
    finally:
        dist.destroy_process_group()


def test_balance_is_contiguous_and_even():
    w = np.array([1, 1, 1, 10, 1, 1, 1, 1, 1, 1, 1, 1])
    cuts = shard.balance(w, 3)
    assert cuts[0] == 0 and cuts[-1] == len(w) and np.all(np.diff(cuts) >= 0)
    sums = [w[cuts[i]:cuts[i + 1]].sum() for i in range(3)]
    assert max(sums) <= 11
    assert list(shard.balance(np.ones(5), 8)[[0, -1]]) == [0, 5]


def test_reads_for_keeps_every_hit():
    reads, regions = _case(1)
    shards = shard.plan_shards(reads, regions, 4)
    assert sorted(np.concatenate(shards).tolist()) == list(range(len(regions)))
    full = _oracle_compute(50)(reads, regions)
    for idx in shards:
        sub = regions[idx]
        m, v = _oracle_compute(50)(shard.reads_for(reads, sub), sub)
        np.testing.assert_array_equal(m, full[0][idx])
        np.testing.assert_array_equal(v, full[1][idx])


def test_gloo_world_size_2():
    reads, regions = _case()
    ref, rv = _oracle_compute(50)(reads, regions)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    sizes = 0
    for rank, out, v, n_mine in res:
        np.testing.assert_array_equal(out, ref)
        np.testing.assert_array_equal(v, rv)
        sizes += n_mine
        assert 0 < n_mine < len(regions)
    assert sizes == len(regions)
    assert (~rv).sum() > 0  # NULL rows (chrUn, no hits) travel through the gather too


@pytest.mark.gpu
def test_gpu_compute_single_rank(gpu):
    """shard.gpu_compute on one GPU (no process group): the full matrix equals the oracle."""
    reads, regions = _case(2)
    ref, rv = _oracle_compute(50)(reads, regions)
    bins = ra.api.Bins([("whole", 50)])
    out, v = shard.profile_sharded(reads, regions, shard.gpu_compute(bins))
    np.testing.assert_array_equal(v, rv)
    np.testing.assert_allclose(out, ref, rtol=1e-12, atol=0)
