"""Test helpers: build C1 inputs for the engine from the committed fixtures, using the
oracle's independent region-window restatement (test infrastructure only)."""
import numpy as np

from oracle import oracle as o
from tests.golden import c1_cases


def c1():
    d = c1_cases.load_inputs()
    S = c1_cases.samples(d)
    G = c1_cases.genome(d)
    E = c1_cases.exons(d)
    return d, S, G, E


def readset(sample, device=0, strand_filter=None):
    from recoup_amd.engine import ReadSet
    chrom = np.zeros(len(sample["start"]), dtype=np.int32)
    return ReadSet(chrom, sample["start"], sample["end"], sample["strand"], sample["seqlengths"], device=device,
                   strand_filter=strand_filter)


def tss_rows(G, flank=(2000, 2000), region="tss"):
    from recoup_amd.engine import RowTable
    s, e = o.regional_ranges(G["start"], G["end"], G["strand"], region, flank)
    chrom = np.zeros(len(s), dtype=np.int32)
    return RowTable.from_ranges(chrom, s, e, G["strand"])


def rna_rows(G, E, flank=(2000, 2000)):
    """coverageRnaRef rows: [upstream flank | exons (list) | downstream flank] per gene."""
    from recoup_amd.engine import RowTable
    f1, f2 = flank
    ls, le = o.promoters(G["start"], G["end"], G["strand"], f1 if f1 else 1, 0)
    rs_, re_ = o.flank_end(G["start"], G["end"], G["strand"], (f2 if f1 else 1))
    seg_off = [0]
    st, en, sd, gr = [], [], [], []
    for i in range(len(G["start"])):
        st.append(ls[i]); en.append(le[i]); sd.append(G["strand"][i]); gr.append(0)
        for j in range(E["seg_off"][i], E["seg_off"][i + 1]):
            st.append(E["start"][j]); en.append(E["end"][j]); sd.append(E["strand"][j]); gr.append(1)
        st.append(rs_[i]); en.append(re_[i]); sd.append(G["strand"][i]); gr.append(2)
        seg_off.append(len(st))
    n = len(st)
    return RowTable(np.array(seg_off), np.zeros(n, np.int32), np.array(st), np.array(en), np.array(sd),
                    seg_group=np.array(gr), group_is_list=np.array([0, 1, 0, 0]))


def unequal_bins(flank, fbs, rbs, stat="mean", interp="auto", scale=1.0):
    """profile.R:13-81 parts: upstream / center / downstream (binned or per-base flanks)."""
    from recoup_amd.engine import Bins
    f1, f2 = flank
    r = np.asarray(flank, dtype=float) / sum(flank)
    parts = []
    if f1:
        parts.append(("upstream", int(np.round(2 * fbs * r[0]))) if fbs else ("upstream", 0, f1))
    parts.append(("center", rbs))
    if f2:
        parts.append(("downstream", int(np.round(2 * fbs * r[1]))) if fbs else ("downstream", 0, f2))
    return Bins(parts, flank=flank, stat=stat, interp=interp, scale=scale)
