"""Region sharding over GPUs: one process per GPU, no data-path collective.

Regions are independent in the reference (cmclapply over mask elements,
R/coverage.R:147-154; one splitVector per row, R/profile.R:198), so the path partitions:
regions sorted by (chromosome, start) are cut into ``world`` contiguous shards balanced by
an estimate of their work (overlapping reads + a per-region constant), and each rank
indexes only the reads that can touch its shard.  The only collective is the optional
reassembly of the R x B matrix after the compute (``gather=``), done once with RCCL (nccl
backend) on GPU ranks or gloo on CPU ranks.
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


def profile_sharded(reads, regions, compute, group=None, gather="all", per_region=64.0):
    """Run ``compute(shard_reads, shard_regions) -> (matrix (n, B) float64, valid (n,) bool)``
    on this rank's shard and, with ``gather="all"``, reassemble the full R x B matrix (region
    order of ``regions``) on every rank with one all_gather.  ``gather=None`` returns only the
    local shard: (indices, matrix, valid)."""
    import torch.distributed as dist

    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    shards = plan_shards(reads, regions, world, per_region)
    mine = shards[rank]
    sub = regions[mine]
    mat, valid = compute(reads_for(reads, sub), sub)
    mat = np.asarray(mat, dtype=np.float64)
    valid = np.asarray(valid, dtype=bool)
    if gather is None or world == 1:
        if world == 1:
            out = np.zeros((len(regions), mat.shape[1]))
            v = np.zeros(len(regions), dtype=bool)
            out[mine], v[mine] = mat, valid
            return out, v
        return mine, mat, valid
    B = int(mat.shape[1]) if mat.ndim == 2 else 0
    nmax = max(len(s) for s in shards)
    backend = dist.get_backend(group)
    dev = torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu")
    # one padded block per rank: B columns of values + 1 column of validity
    blk = torch.zeros((nmax, B + 1), dtype=torch.float64, device=dev)
    if len(mine):
        blk[:len(mine), :B] = torch.from_numpy(mat).to(dev)
        blk[:len(mine), B] = torch.from_numpy(valid.astype(np.float64)).to(dev)
    allb = torch.empty((world, nmax, B + 1), dtype=torch.float64, device=dev)
    if backend == "nccl":
        dist.all_gather_into_tensor(allb, blk, group=group)
    else:
        dist.all_gather(list(allb.unbind(0)), blk, group=group)
    allb = allb.cpu().numpy()
    out = np.zeros((len(regions), B))
    v = np.zeros(len(regions), dtype=bool)
    for r, idx in enumerate(shards):
        out[idx] = allb[r, :len(idx), :B]
        v[idx] = allb[r, :len(idx), B] != 0
    return out, v


def gpu_compute(bins, device=None, ignore_strand=True):
    """The per-rank compute of ``profile_sharded`` on this rank's GPU (HIP engine)."""
    from .api import _readset, _rows_from_mask
    from .engine import Plan

    def run(shard_reads, shard_regions):
        dev = torch.cuda.current_device() if device is None else device
        rs, levels = _readset(shard_reads, dev, None)
        return Plan(rs, _rows_from_mask(shard_regions, levels, ignore_strand), bins).run()
    return run


__all__ = ["balance", "plan_shards", "reads_for", "profile_sharded", "gpu_compute", "GRanges"]
