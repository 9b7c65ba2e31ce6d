"""Region sharding over GPUs: one process per GPU, no data-path collective.

Regions are independent in the reference (cmclapply over mask elements,
R/coverage.R:147-154; one splitVector per row, R/profile.R:198), so the path partitions:
regions sorted by (chromosome, start) are cut into ``world`` contiguous shards balanced by
an estimate of their work (overlapping reads + a per-region constant), and each rank
indexes only the reads that can touch its shard.  The only collective is the optional
reassembly of the R x B matrix after the compute (``gather=``), done once with RCCL (nccl
backend) on device-resident blocks on GPU ranks, or gloo on CPU ranks.
"""
import numpy as np
import torch

from .granges import GRanges


def balance(weights, world):
    """Cut points of ``world`` contiguous chunks with near-equal summed weight."""
    w = np.asarray(weights, dtype=np.float64)
    cum = np.concatenate([[0.0], np.cumsum(w)])
    targets = cum[-1] * np.arange(1, world) / world
    cuts = np.clip(np.searchsorted(cum, targets, side="left"), 1, len(w))
    nearer = (targets - cum[cuts - 1]) < (cum[cuts] - targets)  # nearest prefix sum to each target
    cuts = np.maximum.accumulate(np.where(nearer, cuts - 1, cuts))
    return np.concatenate([[0], cuts, [len(w)]]).astype(np.int64)


def region_order(regions):
    """Regions sorted by (chromosome code, start): the shard order."""
    return np.lexsort((regions.start, regions.seqcodes))


def work_estimate(reads, regions, per_region=64.0):
    """Candidate reads per region (reads of the region's chromosome whose start lies in
    [region.start - max read width + 1, region.end]) plus a per-region constant."""
    est = np.full(len(regions), per_region)
    codes = regions.codes_in(reads.seqlevels)
    maxw = int(reads.width.max()) if len(reads) else 1
    for c in np.unique(codes):
        if c < 0:
            continue
        starts = np.sort(reads.start[reads.seqcodes == c])
        sel = codes == c
        lo = np.searchsorted(starts, regions.start[sel] - maxw + 1, side="left")
        hi = np.searchsorted(starts, regions.end[sel], side="right")
        est[sel] += hi - lo
    return est


def plan_shards(reads, regions, world, per_region=64.0):
    """Per rank: indices (into ``regions``) of its contiguous shard."""
    order = region_order(regions)
    cuts = balance(work_estimate(reads, regions, per_region)[order], world)
    return [order[cuts[r]:cuts[r + 1]] for r in range(world)]


def reads_for(reads, regions):
    """The reads a shard needs: per chromosome, those overlapping [min start, max end] of the
    shard's regions.  A region's coverage depends only on the reads it hits (with NA
    seqlengths its length is the max end of those hits, R/coverage.R:201), so the shard's
    result is unchanged."""
    keep = np.zeros(len(reads), dtype=bool)
    codes = regions.codes_in(reads.seqlevels)
    for c in np.unique(codes):
        if c < 0:
            continue
        sel = codes == c
        lo, hi = regions.start[sel].min(), regions.end[sel].max()
        keep |= (reads.seqcodes == c) & (reads.start <= hi) & (reads.end >= lo)
    return reads[keep]


def profile_sharded(reads, regions, compute, group=None, gather="all", per_region=64.0, as_tensor=False):
    """Run ``compute(shard_reads, shard_regions)`` on this rank's shard and, with
    ``gather="all"``, reassemble the full R x B matrix (region order of ``regions``) on every
    rank with one all_gather.

    ``compute`` returns either ``(matrix (n, B) numpy, valid (n,) bool)`` (host compute, e.g.
    the oracle in CPU tests) or ``(out (B, n) torch tensor, valid (n,) tensor)`` -- the engine's
    R column-major device buffer (``gpu_compute``).  A device result stays in HBM through the
    collective (RCCL over xGMI) and the placement; only the final matrix is copied to the host
    (or returned on the device with ``as_tensor``: shape (B, R), column-major R x B).
    ``gather=None`` returns only the local shard: (indices, matrix, valid)."""
    import torch.distributed as dist

    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    shards = plan_shards(reads, regions, world, per_region)
    mine = shards[rank]
    sub = regions[mine]
    mat, valid = compute(reads_for(reads, sub), sub)
    if isinstance(mat, torch.Tensor):
        cm = mat  # (B, n) column-major
        vt = torch.as_tensor(valid, device=cm.device).to(torch.float64).reshape(1, -1)
    else:
        cm = torch.from_numpy(np.ascontiguousarray(np.asarray(mat, dtype=np.float64).T))
        vt = torch.from_numpy(np.asarray(valid, dtype=np.float64)).reshape(1, -1)
    B = int(cm.shape[0])
    if gather is None and world > 1:
        return mine, cm.T.cpu().numpy() if not as_tensor else cm, vt[0].cpu().numpy() != 0
    backend = dist.get_backend(group) if world > 1 else None
    if backend == "nccl":  # RCCL gathers device tensors: host results are copied across
        dev = torch.device("cuda", torch.cuda.current_device())
    elif backend is None:
        dev = cm.device
    else:
        dev = torch.device("cpu")
    nmax = max(len(s) for s in shards)
    # one padded block per rank: B rows of values + 1 row of validity, columns = the shard's regions
    blk = torch.zeros((B + 1, nmax), dtype=torch.float64, device=dev)
    n = len(mine)
    if n:
        blk[:B, :n].copy_(cm[:, :n])
        blk[B, :n].copy_(vt[0, :n])
    if world > 1:
        allb = torch.empty((world, B + 1, nmax), dtype=torch.float64, device=dev)
        if backend == "nccl":
            dist.all_gather_into_tensor(allb, blk, group=group)
        else:
            dist.all_gather(list(allb.unbind(0)), blk, group=group)
    else:
        allb = blk.unsqueeze(0)
    full = torch.zeros((B + 1, len(regions)), dtype=torch.float64, device=dev)
    for r, idx in enumerate(shards):
        if len(idx):
            full.index_copy_(1, torch.as_tensor(idx, device=dev), allb[r, :, :len(idx)])
    valid_all = (full[B] != 0).cpu().numpy()
    if as_tensor:
        return full[:B], valid_all
    return full[:B].T.cpu().numpy(), valid_all


def gpu_compute(bins, device=None, ignore_strand=True):
    """The per-rank compute of ``profile_sharded`` on this rank's GPU (HIP engine)."""
    from .api import _readset, _rows_from_mask
    from .engine import Plan

    def run(shard_reads, shard_regions):
        dev = torch.cuda.current_device() if device is None else device
        rs, levels = _readset(shard_reads, dev, None)
        plan = Plan(rs, _rows_from_mask(shard_regions, levels, ignore_strand), bins)
        out = plan.empty_output()  # (B, n): the R column-major matrix, stays in HBM
        valid = torch.empty(max(plan.n_rows, 1), dtype=torch.uint8, device=out.device)
        plan.execute(out, valid)
        plan.status()
        return out, valid[:plan.n_rows]
    return run


__all__ = ["balance", "plan_shards", "reads_for", "profile_sharded", "gpu_compute", "GRanges"]
