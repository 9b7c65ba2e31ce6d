"""Synthetic workloads of BASELINE.json configs, generated on the GPU.

Benchmark / test infrastructure (not part of the product path).  Reads come out as device
tensors (chrom int32, start int32, end int32, strand int8), regions as host arrays.  All
draws use a seeded torch generator on the target device, so one seed gives one data set.

  c2: 10k TSS +-2 kb, 200 bins, 10M single-end reads (180 bp): 70 % uniform + 30 % Normal(TSS, 300)
  c4: 200k ChIP peak summits +-1 kb (width-1 "custom" regions), 1000 bins, 200M reads (180 bp):
      30 % within +-500 bp of a summit with Pareto(1.5) per-peak weights (truncated at 1000x
      the median weight), 70 % uniform
  c5: 25k regions x 4000 bp per base, 500M DNase cut fragments (50 bp), 40 % at regions
"""
import numpy as np
import torch

# mm10 chromosome lengths (chr1..chr19, chrX, chrY)
MM10 = np.array([195471971, 182113224, 160039680, 156508116, 151834684, 149736546, 145441459, 129401213,
                 124595110, 130694993, 122082543, 120129022, 120421639, 124902244, 104043685, 98207768,
                 94987271, 90702639, 61431566, 171031299, 91744698], dtype=np.int64)
MM10_NAMES = [f"chr{i}" for i in range(1, 20)] + ["chrX", "chrY"]


def _gen(device, seed):
    g = torch.Generator(device=device)
    g.manual_seed(int(seed))
    return g


def _uniform_positions(n, lens_t, g, device, margin):
    """n positions: chromosome chosen proportional to length, uniform inside [margin, len - margin]."""
    p = lens_t.double() / lens_t.sum()
    cdf = torch.cumsum(p, 0)
    u = torch.rand(n, generator=g, device=device, dtype=torch.float64)
    chrom = torch.searchsorted(cdf, u).clamp_(max=len(lens_t) - 1).to(torch.int32)
    span = (lens_t[chrom.long()] - 2 * margin).double()
    pos = (margin + torch.rand(n, generator=g, device=device, dtype=torch.float64) * span).to(torch.int64)
    return chrom, pos


def _reads(chrom, start, width, g, device):
    n = start.numel()
    strand = torch.randint(0, 2, (n,), generator=g, device=device, dtype=torch.int8)
    s = start.to(torch.int32).clamp_(min=1)
    e = (s + (width - 1)).to(torch.int32)
    return chrom.to(torch.int32), s, e, strand


def _sorted_regions(chrom, pos):
    key = chrom.to(torch.int64) * (1 << 32) + pos
    order = torch.argsort(key)
    return chrom[order], pos[order]


def c4(device="cuda:0", seed=20261015, n_regions=200_000, n_reads=200_000_000, enriched=0.30, width=180,
       flank=1000, n_bins=1000):
    g = _gen(device, seed)
    lens = torch.as_tensor(MM10, device=device)
    pc, pp = _uniform_positions(n_regions, lens, g, device, margin=2500)
    pc, pp = _sorted_regions(pc, pp)
    n_enr = int(n_reads * enriched)
    # Pareto(alpha = 1.5) per-peak weights -> hot regions, truncated at 1000x the median weight
    # (an untruncated draw over 200k peaks can hand one 2 kb peak a third of all reads)
    u = torch.rand(n_regions, generator=g, device=device, dtype=torch.float64)
    w = (1.0 - u).pow(-1.0 / 1.5).clamp_(max=1000.0 * 2.0 ** (1.0 / 1.5))
    cdf = torch.cumsum(w / w.sum(), 0)
    pk = torch.searchsorted(cdf, torch.rand(n_enr, generator=g, device=device, dtype=torch.float64))
    pk = pk.clamp_(max=n_regions - 1)
    off = torch.randint(-500, 501, (n_enr,), generator=g, device=device, dtype=torch.int64)
    ec = pc[pk]
    es = pp[pk] + off - width // 2
    uc, us = _uniform_positions(n_reads - n_enr, lens, g, device, margin=width)
    chrom = torch.cat([ec, uc])
    start = torch.cat([es, us])
    del ec, es, uc, us, pk, off
    reads = _reads(chrom, start, width, g, device)
    # width-1 summits, "custom" region -> promoters(up = flank, down = flank): [p - f, p + f - 1]
    pos = pp.cpu().numpy()
    regions = dict(chrom=pc.cpu().numpy().astype(np.int32), start=(pos - flank).astype(np.int32),
                   end=(pos + flank - 1).astype(np.int32), strand=np.full(n_regions, 2, np.int8))
    return dict(name="c4", reads=reads, seqlen=MM10.copy(), regions=regions, n_bins=n_bins, flank=(flank, flank),
                width=width)


def c2(device="cuda:0", seed=20261015, n_regions=10_000, n_reads=10_000_000, enriched=0.30, width=180,
       flank=2000, n_bins=200):
    g = _gen(device, seed)
    lens = torch.as_tensor(MM10, device=device)
    tc, tp = _uniform_positions(n_regions, lens, g, device, margin=2500)
    tc, tp = _sorted_regions(tc, tp)
    tstrand = torch.randint(0, 2, (n_regions,), generator=g, device=device, dtype=torch.int8)
    n_enr = int(n_reads * enriched)
    k = torch.randint(0, n_regions, (n_enr,), generator=g, device=device)
    off = (torch.randn(n_enr, generator=g, device=device, dtype=torch.float64) * 300).round().to(torch.int64)
    ec, es = tc[k], tp[k] + off - width // 2
    uc, us = _uniform_positions(n_reads - n_enr, lens, g, device, margin=width)
    reads = _reads(torch.cat([ec, uc]), torch.cat([es, us]), width, g, device)
    pos = tp.cpu().numpy()
    st = tstrand.cpu().numpy()
    # promoters(up = f1, down = f2) of a TSS p: '+' [p - f1, p + f2 - 1]; '-' [p - f2 + 1, p + f1]
    s = np.where(st == 1, pos - flank + 1, pos - flank)
    e = np.where(st == 1, pos + flank, pos + flank - 1)
    regions = dict(chrom=tc.cpu().numpy().astype(np.int32), start=s.astype(np.int32), end=e.astype(np.int32),
                   strand=st.astype(np.int8))
    return dict(name="c2", reads=reads, seqlen=MM10.copy(), regions=regions, n_bins=n_bins, flank=(flank, flank),
                width=width)


def c5(device="cuda:0", seed=20261015, n_regions=25_000, n_reads=500_000_000, enriched=0.40, width=50,
       flank=2000):
    d = c2(device=device, seed=seed, n_regions=n_regions, n_reads=n_reads, enriched=enriched, width=width,
           flank=flank, n_bins=0)
    d["name"] = "c5"
    return d


def n_overlaps(reads, regions, width, device="cuda:0"):
    """Exact per-region overlap counts (fixed-width reads): binary search on the sorted starts of
    each (chromosome) -- the harness's independent count of n_ovl."""
    chrom, start, _, _ = reads
    key = chrom.to(torch.int64) * (1 << 32) + start.to(torch.int64)
    ks, _ = torch.sort(key)
    rc = torch.as_tensor(regions["chrom"], device=device, dtype=torch.int64)
    lo = rc * (1 << 32) + torch.as_tensor(regions["start"], device=device, dtype=torch.int64) - (width - 1)
    hi = rc * (1 << 32) + torch.as_tensor(regions["end"], device=device, dtype=torch.int64)
    cnt = torch.searchsorted(ks, hi, right=True) - torch.searchsorted(ks, lo, right=False)
    return cnt.cpu().numpy()
