"""C1 configuration (BASELINE.json configs[0]) built from the reference's own fixture.

The cases follow the reference's own tests and man-page examples:
  tss_*   inst/unitTests/test_recoup.R:4-13 (TSS +-2000, per-base) + the forced
          heatmap binning pass recoup.R:659-671 (forcedBinSize[2] = 200)
  tss150  man/profileMatrix.Rd:32-50 (TSS, regionBinSize = 150 -> RNG bin layout)
  gb_*    inst/unitTests/test_recoup.R:15-26 (genebody, flankBinSize 50, regionBinSize 150)
  rna     man/coverageRnaRef.Rd:60-68 (test.exons GRangesList + helper genes)
  calc    man/calcCoverage.Rd:47-55 (calcCoverage over whole genes; stored as checksums)

``compute_all_with_oracle`` evaluates every case with the CPU oracle; make_fixtures.py
commits the result as c1_expected.npz.
"""
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
STRAND = {"+": 0, "-": 1, "*": 2}


def load_inputs():
    d = np.load(os.path.join(HERE, "recoup_test_data.npz"))
    return {k: d[k] for k in d.files}


def samples(d):
    out = []
    for i in range(2):
        out.append(dict(id=str(d[f"s{i}_id"]), name=str(d[f"s{i}_name"]),
                        start=d[f"s{i}_start"], end=d[f"s{i}_end"], strand=d[f"s{i}_strand"],
                        seqlevels=list(d[f"s{i}_seqlevels"]), seqlengths=d[f"s{i}_seqlengths"]))
    return out


def genome(d):
    return dict(chrom=np.array(d["genome_chromosome"]), start=d["genome_start"].astype(np.int64),
                end=d["genome_end"].astype(np.int64),
                strand=np.array([STRAND[s] for s in d["genome_strand"]], dtype=np.int8),
                names=np.array(d["genome_gene_name"]))


def exons(d):
    ends = d["exons_part_end"]
    off = np.zeros(len(ends) + 1, dtype=np.int64)
    off[1:] = ends
    return dict(seg_off=off, chrom=np.array(d["exons_seqnames"]), start=d["exons_start"].astype(np.int64),
                end=d["exons_end"].astype(np.int64), strand=d["exons_strand"], names=np.array(d["exons_part_names"]))


def compute_all_with_oracle(nthreads=8):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
    from oracle import oracle as o

    d = load_inputs()
    S = samples(d)
    G = genome(d)
    E = exons(d)
    levels = S[0]["seqlevels"]
    chrom_code = {c: i for i, c in enumerate(levels)}
    idx = []
    for s in S:
        chrom = np.zeros(len(s["start"]), dtype=np.int32)  # all reads are on chr12
        idx.append(o.Index(chrom, s["start"], s["end"], s["strand"], s["seqlengths"]))
    gchrom = np.array([chrom_code.get(c, -1) for c in G["chrom"]], dtype=np.int32)
    res = {}

    def cov_of(mask):
        return [o.coverage(ix, mask, True, nthreads) for ix in idx]

    # --- TSS +-2000 (test_recoup.R:4-13) -------------------------------------------
    s, e = o.regional_ranges(G["start"], G["end"], G["strand"], "tss", (2000, 2000))
    tss = o.Mask.from_ranges(gchrom, s, e, G["strand"])
    covs = cov_of(tss)
    base = o.profile_matrix(covs, (2000, 2000), dict(regionBinSize=0, flankBinSize=0))
    heat = o.profile_matrix(covs, (2000, 2000), dict(regionBinSize=200, flankBinSize=0))
    b150 = o.profile_matrix(covs, (2000, 2000), dict(regionBinSize=150, flankBinSize=50))
    for k in range(2):
        res[f"tss_base_s{k}"] = base[k].astype(np.int32)
        res[f"tss_heat_s{k}"] = heat[k]
        res[f"tss150_s{k}"] = b150[k]
        res[f"tss_valid_s{k}"] = np.array([c is not None for c in covs[k]], dtype=np.uint8)

    # --- genebody (test_recoup.R:15-26) ------------------------------------------
    s, e = o.regional_ranges(G["start"], G["end"], G["strand"], "genebody", (2000, 2000))
    gb = o.Mask.from_ranges(gchrom, s, e, G["strand"])
    covs = cov_of(gb)
    for stat in ("mean", "median"):
        prof = o.profile_matrix(covs, (2000, 2000),
                                dict(regionBinSize=150, flankBinSize=50, sumStat=stat))
        for k in range(2):
            res[f"gb_{stat}_s{k}"] = prof[k]
    for k in range(2):
        res[f"gb_valid_s{k}"] = np.array([c is not None for c in covs[k]], dtype=np.uint8)

    # --- RNA (coverageRnaRef.Rd) ----------------------------------------------------
    # coverageRnaRef flanks come from helperRanges in helper order; exons in list order.
    ex = o.Mask(E["seg_off"], np.array([chrom_code.get(c, -1) for c in E["chrom"]], dtype=np.int32),
                E["start"], E["end"], E["strand"])
    ls, le = o.promoters(G["start"], G["end"], G["strand"], 2000, 0)
    rs, re_ = o.flank_end(G["start"], G["end"], G["strand"], 2000)
    left = o.Mask.from_ranges(gchrom, ls, le, G["strand"])
    right = o.Mask.from_ranges(gchrom, rs, re_, G["strand"])
    rcov = []
    for ix in idx:
        rcov.append(o.rna_merge(o.coverage(ix, left, True, nthreads), o.coverage(ix, ex, True, nthreads),
                                o.coverage(ix, right, True, nthreads)))
    prof = o.profile_matrix(rcov, (2000, 2000), dict(regionBinSize=150, flankBinSize=50))
    for k in range(2):
        res[f"rna_s{k}"] = prof[k]
        res[f"rna_valid_s{k}"] = np.array([c is not None for c in rcov[k]], dtype=np.uint8)

    # --- calcCoverage over whole genes (calcCoverage.Rd) -> checksums ----------------
    whole = o.Mask.from_ranges(gchrom, G["start"], G["end"], G["strand"])
    cc = o.coverage(idx[0], whole, True, nthreads)
    res["calc_len"] = np.array([len(c) if c is not None else -1 for c in cc], dtype=np.int64)
    res["calc_sum"] = np.array([int(c.sum()) if c is not None else 0 for c in cc], dtype=np.int64)
    res["calc_wsum"] = np.array([int((c.astype(np.int64) * (np.arange(len(c)) % 9973)).sum())
                                 if c is not None else 0 for c in cc], dtype=np.int64)
    return res
