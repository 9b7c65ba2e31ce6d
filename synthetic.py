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


def _sample_seed(seed, sample):
    """Seed of sample k's reads (k > 0): the same regions, an independent read set."""
    return (int(seed) * 1_000_003 + 7_919 * int(sample)) % (2 ** 63)


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
       flank=1000, n_bins=1000, sample=0):
    """``sample`` k > 0: the same regions, another sample's reads (its own peak heights and
    draws) -- what profileMatrix loops over (R/profile.R:13-98)."""
    g = _gen(device, seed)
    lens = torch.as_tensor(MM10, device=device)
    pc, pp = _uniform_positions(n_regions, lens, g, device, margin=2500)
    pc, pp = _sorted_regions(pc, pp)
    if sample:
        g = _gen(device, _sample_seed(seed, sample))
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
       flank=2000, n_bins=200, sample=0):
    g = _gen(device, seed)
    lens = torch.as_tensor(MM10, device=device)
    tc, tp = _uniform_positions(n_regions, lens, g, device, margin=2500)
    tc, tp = _sorted_regions(tc, tp)
    tstrand = torch.randint(0, 2, (n_regions,), generator=g, device=device, dtype=torch.int8)
    if sample:
        g = _gen(device, _sample_seed(seed, sample))
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
       flank=2000, sample=0):
    d = c2(device=device, seed=seed, n_regions=n_regions, n_reads=n_reads, enriched=enriched, width=width,
           flank=flank, n_bins=0, sample=sample)
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


def c3(device="cuda:0", seed=20261015, n_genes=25_000, n_pairs=50_000_000, width=100, exonic=0.70,
       flank=2000, region_bins=500, flank_bins=50, short_frac=0.05, genome=None, sample=0):
    """coverageRnaRef spliced (C3): genes of 1 + Poisson(8) exons (lognormal widths, median 150 bp;
    lognormal introns, median 2 kb; ~5 % of genes with < 500 exonic bp -> interpolated centres),
    2 x n_pairs mate alignments of `width` bp (mates read independently, R/ranges.R:117-120),
    `exonic` of them drawn along transcripts -- those crossing an exon junction are split into
    two blocks (spliceAction "split") -- the rest uniform.  Rows: c(upstream flank, exon list,
    downstream flank) per gene, flank bins 50 / centre 500 bins."""
    lens_np = MM10 if genome is None else np.asarray(genome, dtype=np.int64)
    rng = np.random.default_rng(seed)
    n_ex = 1 + rng.poisson(8, n_genes)
    short = rng.random(n_genes) < short_frac
    n_ex[short] = rng.integers(1, 3, short.sum())
    tot = int(n_ex.sum())
    ew = np.maximum(np.round(rng.lognormal(np.log(150), 0.6, tot)), 20).astype(np.int64)
    gi = np.repeat(np.arange(n_genes), n_ex)
    ew[short[gi]] = np.minimum(ew[short[gi]], 200)
    iw = np.maximum(np.round(rng.lognormal(np.log(2000), 1.0, tot)), 50).astype(np.int64)
    first = np.zeros(n_genes + 1, np.int64)
    first[1:] = np.cumsum(n_ex)
    iw[first[1:] - 1] = 0  # no intron after a gene's last exon
    span = np.add.reduceat(ew + iw, first[:-1])
    chrom = rng.choice(len(lens_np), n_genes, p=lens_np / lens_np.sum()).astype(np.int32)
    gstart = (flank + 10 + rng.random(n_genes) * (lens_np[chrom] - span - 2 * flank - 20)).astype(np.int64)
    order = np.lexsort((gstart, chrom))
    chrom, gstart, n_ex2, span = chrom[order], gstart[order], n_ex[order], span[order]
    # exon coordinates in sorted gene order
    ex_s, ex_e, ex_gene = [], [], []
    for new, old in enumerate(order):
        w = ew[first[old]:first[old + 1]]
        gaps = iw[first[old]:first[old + 1]]
        st = gstart[new] + np.concatenate([[0], np.cumsum(w + gaps)[:-1]])
        ex_s.append(st)
        ex_e.append(st + w - 1)
        ex_gene.append(np.full(len(w), new))
    ex_s, ex_e, ex_gene = np.concatenate(ex_s), np.concatenate(ex_e), np.concatenate(ex_gene)
    seg_off = np.zeros(n_genes + 1, np.int64)
    seg_off[1:] = np.cumsum(n_ex2)
    gstrand = rng.integers(0, 2, n_genes).astype(np.int8)
    gend = ex_e[seg_off[1:] - 1]
    # ---- reads on the GPU (sample k > 0: the same genes, another sample's reads)
    g = _gen(device, seed if not sample else _sample_seed(seed, sample))
    n = 2 * n_pairs
    n_ex_reads = int(n * exonic)
    dev = device
    exlen_g = torch.as_tensor(np.add.reduceat(ex_e - ex_s + 1, seg_off[:-1]), device=dev)
    cum = torch.as_tensor(np.concatenate([[0], np.cumsum(ex_e - ex_s + 1)]), device=dev)  # flat transcript coords
    t_s = torch.as_tensor(ex_s, device=dev)
    t_e = torch.as_tensor(ex_e, device=dev)
    gsel = torch.randint(0, n_genes, (n_ex_reads,), generator=g, device=dev)
    base = cum[torch.as_tensor(seg_off[:-1], device=dev)][gsel]
    room = (exlen_g[gsel] - width).clamp_(min=0)
    t = base + (torch.rand(n_ex_reads, generator=g, device=dev, dtype=torch.float64) * (room + 1)).to(torch.int64)
    k = (torch.searchsorted(cum, t, right=True) - 1).clamp_(max=len(ex_s) - 1)
    gs = t_s[k] + (t - cum[k])
    left = t_e[k] - gs + 1  # bases to the end of exon k
    last = torch.as_tensor(seg_off[1:] - 1, device=dev)[gsel]
    split = (left < width) & (k < last)
    b1e = torch.where(split, t_e[k], gs + width - 1)
    kn = (k + 1).clamp_(max=len(ex_s) - 1)
    b2s = t_s[kn][split]
    b2e = b2s + (width - left[split]) - 1
    gch = torch.as_tensor(chrom, device=dev)[torch.as_tensor(ex_gene, device=dev)[k]]
    uc, us = _uniform_positions(n - n_ex_reads, torch.as_tensor(lens_np, device=dev), g, dev, margin=width)
    c_all = torch.cat([gch, gch[split], uc.to(gch.dtype)])
    s_all = torch.cat([gs, b2s, us])
    e_all = torch.cat([b1e, b2e, us + width - 1])
    st = torch.randint(0, 2, (c_all.numel(),), generator=g, device=dev, dtype=torch.int8)
    reads = (c_all.to(torch.int32), s_all.clamp(min=1).to(torch.int32), e_all.to(torch.int32), st)
    genes = dict(chrom=chrom, start=gstart.astype(np.int64), end=gend.astype(np.int64), strand=gstrand)
    exons = dict(seg_off=seg_off, chrom=chrom[ex_gene], start=ex_s, end=ex_e, strand=gstrand[ex_gene])
    return dict(name="c3", reads=reads, seqlen=lens_np.copy(), genes=genes, exons=exons, flank=(flank, flank),
                region_bins=region_bins, flank_bins=flank_bins, n_split=int(split.sum()), width=width)


def rna_rows(d, ignore_strand=True):
    """coverageRnaRef rows of a c3 data set: [upstream flank | exons (list) | downstream flank]."""
    from recoup_amd.engine import RowTable
    G, E = d["genes"], d["exons"]
    f1, f2 = d["flank"]
    n = len(G["start"])
    minus = G["strand"] == 1
    # promoters(up = f1, down = 0) and flank(width = f2, start = FALSE) of the gene
    ls = np.where(minus, G["end"] + 1, G["start"] - f1)
    le = np.where(minus, G["end"] + f1, G["start"] - 1)
    rs = np.where(minus, G["start"] - f2, G["end"] + 1)
    re_ = np.where(minus, G["start"] - 1, G["end"] + f2)
    cnt = np.diff(E["seg_off"]) + 2
    seg_off = np.zeros(n + 1, np.int64)
    seg_off[1:] = np.cumsum(cnt)
    m = int(seg_off[-1])
    first, lastp = seg_off[:-1], seg_off[1:] - 1
    inner = np.ones(m, bool)
    inner[first] = False
    inner[lastp] = False
    ch = np.empty(m, np.int32); s = np.empty(m, np.int64); e = np.empty(m, np.int64)
    st = np.empty(m, np.int8); grp = np.ones(m, np.int8)
    ch[first], s[first], e[first], st[first], grp[first] = G["chrom"], ls, le, G["strand"], 0
    ch[lastp], s[lastp], e[lastp], st[lastp], grp[lastp] = G["chrom"], rs, re_, G["strand"], 2
    ch[inner], s[inner], e[inner], st[inner] = E["chrom"], E["start"], E["end"], E["strand"]
    return RowTable(seg_off, ch, s.astype(np.int32), e.astype(np.int32), st, seg_group=grp,
                    group_is_list=np.array([0, 1, 0, 0], np.uint8), ignore_strand=ignore_strand)


def n_overlaps_segments(reads, seg_chrom, seg_start, seg_end, device="cuda:0"):
    """Reads overlapping each segment, any widths: #(start <= e) - #(end < s) on one chromosome."""
    chrom, start, end, _ = reads
    ks, _ = torch.sort(chrom.to(torch.int64) * (1 << 32) + start.to(torch.int64))
    ke, _ = torch.sort(chrom.to(torch.int64) * (1 << 32) + end.to(torch.int64))
    c = torch.as_tensor(seg_chrom, device=device, dtype=torch.int64) * (1 << 32)
    s = c + torch.as_tensor(seg_start, device=device, dtype=torch.int64)
    e = c + torch.as_tensor(seg_end, device=device, dtype=torch.int64)
    a = torch.searchsorted(ks, e, right=True) - torch.searchsorted(ks, c, right=False)
    b = torch.searchsorted(ke, s, right=False) - torch.searchsorted(ke, c, right=False)
    return (a - b).cpu().numpy()
