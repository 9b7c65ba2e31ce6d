"""Evaluate the oracle on an engine RowTable + Bins (test infrastructure).

A row is c(cov(g0), cov(g1), ...) over its groups (R/coverage.R:115-121 for coverageRnaRef);
each group's coverage is the oracle's coverageFromRanges of that mask element.  The profile
is then binned part by part with the oracle's splitVector (R/profile.R slices)."""
import numpy as np

from oracle import oracle as o

WHERE = {0: "whole", 1: "center", 2: "upstream", 3: "downstream"}
STAT = {0: "mean", 1: "median"}
INTERP = {0: "auto", 1: "spline", 2: "linear", 3: "neighborhood"}


def index_for(reads, seqlen, strand_filter=None):
    chrom, start, end, strand = reads
    return o.Index(chrom, start, end, strand, seqlen, strand_filter=strand_filter)


def row_coverage(ix, rows):
    """Per-row coverage vectors (None = the reference's NULL)."""
    groups = rows.seg_group if rows.seg_group is not None else np.zeros(len(rows.start), np.int8)
    per_group = {}
    for g in range(4):
        sel_rows, off, segs = [], [0], []
        for r in range(rows.n_rows):
            js = [j for j in range(rows.seg_off[r], rows.seg_off[r + 1]) if groups[j] == g]
            if js:
                sel_rows.append(r)
                segs.extend(js)
                off.append(len(segs))
        if not sel_rows:
            continue
        segs = np.array(segs)
        m = o.Mask(np.array(off), rows.chrom[segs], rows.start[segs], rows.end[segs], rows.strand[segs])
        cov = o.coverage(ix, m, rows.ignore_strand)
        per_group[g] = dict(zip(sel_rows, cov))
    out = []
    for r in range(rows.n_rows):
        parts = [per_group[g][r] for g in sorted(per_group) if r in per_group[g]]
        if not parts or any(p is None for p in parts):
            out.append(None)
        else:
            out.append(np.concatenate(parts))
    return out


def profile(cov, bins, kind="Rejection"):
    """Expected matrix and validity for an engine Bins spec."""
    mats = []
    f = bins.flank
    for wh, nb, width in zip(bins.where, bins.n_bins, bins.width):
        where = WHERE[int(wh)]
        if nb == 0:
            rows = []
            for x in cov:
                if x is None:
                    rows.append(np.zeros(width))
                    continue
                v = x.astype(np.float64) * bins.scale
                v = _slice(v, where, f)
                rows.append(v)
            mats.append(o._rbind(rows))
        else:
            mats.append(o._bin_matrix(cov, int(nb), STAT[bins.stat], INTERP[bins.interp],
                                      None if where == "whole" else f, where, bins.scale, kind))
    valid = np.array([x is not None for x in cov])
    return np.hstack(mats), valid


def _slice(v, where, f):
    L = len(v)
    if where == "center":
        return v[f[0]:L - f[1]]
    if where == "upstream":
        return v[:f[0]]
    if where == "downstream":
        return v[L - f[1]:]
    return v
