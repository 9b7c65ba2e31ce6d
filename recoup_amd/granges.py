"""Host-side genomic ranges: the slice of GenomicRanges the hot path's callers use.

``GRanges``      seqnames / 1-based closed [start, end] / strand / names / seqlengths, held as
                 numpy columns (chromosomes as integer codes into ``seqlevels``).
``GRangesList``  a partitioning of one flat GRanges (``offsets``), e.g. the exons of genes.
Window helpers mirror the reference's region construction (R/ranges.R:67-100) and the
GenomicRanges verbs it calls (promoters / resize / flank).  All of this is table
construction on the host; nothing here touches reads.
"""
import numpy as np

STRAND_CODE = {"+": 0, "-": 1, "*": 2}
STRAND_CHAR = np.array(["+", "-", "*"])


def _strand_codes(strand, n):
    if strand is None:
        return np.full(n, 2, dtype=np.int8)
    a = np.asarray(strand)
    if a.dtype.kind in "USO":
        try:
            a = np.array([STRAND_CODE[str(s)] for s in a.ravel()], dtype=np.int8)
        except KeyError as e:
            raise ValueError(f"invalid strand {e}: use '+', '-' or '*'") from None
    a = np.ascontiguousarray(a, dtype=np.int8)
    if a.ndim == 0:
        a = np.full(n, int(a), dtype=np.int8)
    if a.shape[0] != n or (a.size and (a.min() < 0 or a.max() > 2)):
        raise ValueError("strand must be '+', '-', '*' (or codes 0, 1, 2), one per range")
    return a


class GRanges:
    """A GenomicRanges::GRanges restricted to what the coverage/profile path reads."""

    def __init__(self, seqnames, start, end=None, strand=None, names=None, seqlengths=None, width=None,
                 seqlevels=None):
        start = np.asarray(start, dtype=np.int64).ravel()
        n = start.shape[0]
        if end is None:
            if width is None:
                raise ValueError("give end or width")
            end = start + np.asarray(width, dtype=np.int64) - 1
        end = np.broadcast_to(np.asarray(end, dtype=np.int64), (n,)).copy()
        sn = np.asarray(seqnames)
        if sn.ndim == 0:
            sn = np.full(n, sn)
        if sn.dtype.kind in "iu" and seqlevels is not None:
            codes = sn.astype(np.int32)
            levels = list(seqlevels)
        else:
            sn = sn.astype(str)
            if seqlevels is None:
                levels = list(dict.fromkeys(sn.tolist()))
            else:
                levels = list(seqlevels)
            lut = {c: i for i, c in enumerate(levels)}
            try:
                codes = np.array([lut[c] for c in sn.tolist()], dtype=np.int32)
            except KeyError as e:
                raise ValueError(f"seqname {e} not in seqlevels") from None
        if codes.shape[0] != n:
            raise ValueError("seqnames and start differ in length")
        self.seqlevels = levels
        self.seqcodes = codes
        self.start = start
        self.end = end
        self.strand = _strand_codes(strand, n)
        self.names = None if names is None else np.asarray(names).astype(str)
        sl = np.full(len(levels), -1, dtype=np.int64)  # -1 = NA
        if isinstance(seqlengths, dict):
            for k, v in seqlengths.items():
                if k in levels and v is not None:
                    sl[levels.index(k)] = int(v)
        elif seqlengths is not None:
            a = np.asarray(seqlengths, dtype=np.float64)
            sl[:] = np.where(np.isnan(a), -1, a).astype(np.int64)
        self.seqlengths = sl

    # ------------------------------------------------------------------ basics
    def __len__(self):
        return int(self.start.shape[0])

    @property
    def width(self):
        return self.end - self.start + 1

    @property
    def seqnames(self):
        return np.array(self.seqlevels, dtype=object)[self.seqcodes] if len(self) else np.array([], dtype=object)

    def __getitem__(self, idx):
        idx = np.arange(len(self))[idx] if not isinstance(idx, np.ndarray) or idx.dtype != bool else np.nonzero(idx)[0]
        idx = np.atleast_1d(idx)
        return self._like(self.start[idx], self.end[idx], self.strand[idx], self.seqcodes[idx],
                          None if self.names is None else self.names[idx])

    def _like(self, start, end, strand=None, codes=None, names=None):
        g = GRanges.__new__(GRanges)
        g.seqlevels = self.seqlevels
        g.seqcodes = self.seqcodes if codes is None else codes
        g.start = np.asarray(start, dtype=np.int64)
        g.end = np.asarray(end, dtype=np.int64)
        g.strand = self.strand if strand is None else strand
        g.names = self.names if names is None else names
        g.seqlengths = self.seqlengths
        return g

    def codes_in(self, levels):
        """Chromosome codes of these ranges in another level list (-1 = absent there)."""
        lut = {c: i for i, c in enumerate(levels)}
        remap = np.array([lut.get(c, -1) for c in self.seqlevels] + [-1], dtype=np.int32)
        return remap[self.seqcodes]

    def keep_strand(self, strand):
        """``input[strand(input) == strand]`` (R/coverage.R:141-144)."""
        return self[self.strand == STRAND_CODE[strand]]

    def __repr__(self):
        return f"GRanges({len(self)} ranges on {len(self.seqlevels)} seqlevels)"


class GRangesList:
    """GRangesList as (flat GRanges, offsets): element i is flat[offsets[i]:offsets[i+1]]."""

    def __init__(self, flat, offsets, names=None):
        self.flat = flat
        self.offsets = np.ascontiguousarray(offsets, dtype=np.int64)
        if self.offsets[0] != 0 or self.offsets[-1] != len(flat) or np.any(np.diff(self.offsets) < 0):
            raise ValueError("offsets must partition the flat ranges")
        self.names = None if names is None else np.asarray(names).astype(str)

    @classmethod
    def from_list(cls, elements, names=None):
        levels = list(dict.fromkeys(l for g in elements for l in g.seqlevels))
        seq = np.concatenate([np.array(g.seqlevels, dtype=object)[g.seqcodes] for g in elements]) if elements else []
        flat = GRanges(np.asarray(seq, dtype=str), np.concatenate([g.start for g in elements]),
                       np.concatenate([g.end for g in elements]), np.concatenate([g.strand for g in elements]),
                       seqlevels=levels)
        off = np.zeros(len(elements) + 1, dtype=np.int64)
        off[1:] = np.cumsum([len(g) for g in elements])
        return cls(flat, off, names)

    def __len__(self):
        return len(self.offsets) - 1

    def __getitem__(self, i):
        return self.flat[np.arange(self.offsets[i], self.offsets[i + 1])]


# ---------------------------------------------------------------------- GenomicRanges verbs
def promoters(gr, upstream, downstream):
    """GenomicRanges::promoters: '+'/'*' -> [start-up, start+down-1]; '-' -> [end-down+1, end+up]."""
    minus = gr.strand == 1
    s = np.where(minus, gr.end - downstream + 1, gr.start - upstream)
    e = np.where(minus, gr.end + upstream, gr.start + downstream - 1)
    return gr._like(s, e)


def resize(gr, width, fix="start"):
    """GenomicRanges::resize with fix = "start" | "end" (strand-aware)."""
    width = np.broadcast_to(np.asarray(width, dtype=np.int64), (len(gr),))
    minus = gr.strand == 1
    anchor_start = ~minus if fix == "start" else minus
    s = np.where(anchor_start, gr.start, gr.end - width + 1)
    e = np.where(anchor_start, gr.start + width - 1, gr.end)
    return gr._like(s, e)


def flank(gr, width, start=True, both=False):
    """GenomicRanges::flank (both = FALSE): the `width` bases before start / after end."""
    if both:
        raise NotImplementedError("flank(both=TRUE) is not used by the coverage path")
    minus = gr.strand == 1
    at_start = ~minus if start else minus
    s = np.where(at_start, gr.start - width, gr.end + 1)
    e = np.where(at_start, gr.start - 1, gr.end + width)
    return gr._like(s, e)


def getRegionalRanges(ranges, region, flank_):
    """R/ranges.R:67-91."""
    f1, f2 = int(flank_[0]), int(flank_[1])
    if region == "tss":
        return promoters(ranges, f1, f2)
    if region == "tes":
        return promoters(resize(ranges, 1, fix="end"), f1, f2)
    if region == "custom" and np.all(ranges.width == 1):
        return promoters(ranges, f1, f2)
    if region in ("genebody", "custom"):
        w = ranges.width
        return resize(promoters(ranges, f1, 0), w + f1 + f2)
    raise ValueError(f"region must be tss, tes, genebody or custom, not {region!r}")


def getFlankingRanges(ranges, flank_, dir="upstream"):
    """R/ranges.R:93-100."""
    if dir == "upstream":
        return promoters(ranges, flank_, 0)
    if dir == "downstream":
        return flank(ranges, flank_, start=False)
    raise ValueError(dir)
