"""Minimal reader for R's XDR serialization (``save()`` / ``.rda`` files, format 2/3).

Test infrastructure only: used by ``make_fixtures.py`` to turn the reference's own
fixture ``data/recoup_test_data.rda`` into plain ``.npz`` vectors.  It parses data,
never evaluates anything from the file (closures/bytecode are decoded as inert
records).  Follows the public description of R's serialize.c format: a flags word
(type | object bit | attr bit | tag bit | gp levels), reference table for
SYMSXP/ENVSXP/namespace records, ALTREP wrappers for compact sequences.
"""
import gzip
import struct

import numpy as np

NILVALUE, GLOBALENV, UNBOUNDVALUE, MISSINGARG, BASENAMESPACE = 254, 253, 252, 251, 250
NAMESPACESXP, PACKAGESXP, PERSISTSXP, CLASSREFSXP, GENERICREFSXP = 249, 248, 247, 246, 245
BCREPDEF, BCREPREF, EMPTYENV, BASEENV, ATTRLANGSXP, ATTRLISTSXP, ALTREP = 244, 243, 242, 241, 240, 239, 238
REFSXP = 255
NA_INT = -2147483648


class RObj:
    """A decoded R object: ``type`` (SEXPTYPE), ``value`` and ``attr`` (dict)."""

    __slots__ = ("type", "value", "attr")

    def __init__(self, type_, value=None, attr=None):
        self.type = type_
        self.value = value
        self.attr = attr or {}

    def a(self, name):
        v = self.attr.get(name)
        # S4 slots holding NULL are serialized as the symbol "\001NULL\001"
        return None if isinstance(v, _Sym) else v

    @property
    def cls(self):
        c = self.attr.get("class")
        return list(c.value) if c is not None else []

    def __repr__(self):
        v = self.value
        if isinstance(v, np.ndarray):
            v = f"array{v.shape}"
        elif isinstance(v, list):
            v = f"list[{len(v)}]"
        return f"RObj(type={self.type}, cls={self.cls}, value={v})"


class _Sym:
    __slots__ = ("name",)

    def __init__(self, name):
        self.name = name

    def __repr__(self):
        return f"Sym({self.name})"


class _Reader:
    def __init__(self, buf):
        self.b = buf
        self.p = 0
        self.refs = []

    def int(self):
        v = struct.unpack_from(">i", self.b, self.p)[0]
        self.p += 4
        return v

    def length(self):
        n = self.int()
        if n == -1:
            hi, lo = self.int(), self.int()
            n = (hi << 32) + lo
        return n

    def ints(self, n):
        v = np.frombuffer(self.b, dtype=">i4", count=n, offset=self.p).astype(np.int32)
        self.p += 4 * n
        return v

    def reals(self, n):
        v = np.frombuffer(self.b, dtype=">f8", count=n, offset=self.p).astype(np.float64)
        self.p += 8 * n
        return v

    def bytes_(self, n):
        v = self.b[self.p:self.p + n]
        self.p += n
        return v

    def item(self):
        flags = self.int()
        t = flags & 0xFF
        has_attr = bool(flags & (1 << 9))
        has_tag = bool(flags & (1 << 10))
        if t == NILVALUE:
            return None
        if t in (GLOBALENV, UNBOUNDVALUE, MISSINGARG, BASENAMESPACE, EMPTYENV, BASEENV):
            return RObj(t)
        if t == REFSXP:
            idx = flags >> 8
            if idx == 0:
                idx = self.int()
            return self.refs[idx - 1]
        if t in (PERSISTSXP, PACKAGESXP, NAMESPACESXP):
            self.int()  # 0
            n = self.int()
            v = RObj(t, [self.item() for _ in range(n)])
            self.refs.append(v)
            return v
        if t == 1:  # SYMSXP
            s = self.item()
            v = _Sym(s.value if isinstance(s, RObj) else s)
            self.refs.append(v)
            return v
        if t == 4:  # ENVSXP
            self.int()  # locked
            env = RObj(4, {})
            self.refs.append(env)
            enclos = self.item()
            frame = self.item()
            hashtab = self.item()
            attr = self.item()
            env.value = {"enclos": enclos, "frame": frame, "hashtab": hashtab}
            env.attr = self._attrs(attr)
            return env
        if t in (2, 3, 5, 6, 17, ATTRLANGSXP, ATTRLISTSXP):  # pairlist-like
            attr = self.item() if has_attr else None
            tag = self.item() if has_tag else None
            car = self.item()
            cdr = self.item()
            node = RObj(2 if t in (2, ATTRLISTSXP) else t, [(tag, car)], self._attrs(attr))
            if isinstance(cdr, RObj) and cdr.type == 2 and isinstance(cdr.value, list):
                node.value.extend(cdr.value)
            return node
        if t == 9:  # CHARSXP
            n = self.int()
            if n == -1:
                return None
            return self.bytes_(n).decode("utf-8", "replace")
        if t in (10, 13):  # LGLSXP / INTSXP
            n = self.length()
            v = RObj(t, self.ints(n))
        elif t == 14:
            n = self.length()
            v = RObj(t, self.reals(n))
        elif t == 15:
            n = self.length()
            v = RObj(t, self.reals(2 * n))
        elif t == 16:  # STRSXP
            n = self.length()
            v = RObj(t, [self.item() for _ in range(n)])
        elif t in (19, 20):  # VECSXP / EXPRSXP
            n = self.length()
            v = RObj(t, [self.item() for _ in range(n)])
        elif t == 24:  # RAWSXP
            n = self.length()
            v = RObj(t, self.bytes_(n))
        elif t == 25:  # S4SXP
            v = RObj(t, None)
        elif t == ALTREP:
            info = self.item()
            state = self.item()
            attr = self.item()
            return self._altrep(info, state, attr)
        elif t == 22:  # EXTPTRSXP
            v = RObj(t)
            self.refs.append(v)
            v.value = (self.item(), self.item())
        elif t == 23:  # WEAKREFSXP
            v = RObj(t)
            self.refs.append(v)
        elif t == 21:  # BCODESXP: decode as opaque, never executed
            raise NotImplementedError("bytecode objects are not expected in data fixtures")
        else:
            raise ValueError(f"unsupported SEXPTYPE {t} at offset {self.p}")
        if has_attr:
            v.attr = self._attrs(self.item())
        return v

    def _attrs(self, pl):
        out = {}
        if isinstance(pl, RObj) and pl.type == 2:
            for tag, car in pl.value:
                name = tag.name if isinstance(tag, _Sym) else str(tag)
                out[name] = car
        return out

    def _altrep(self, info, state, attr):
        cls = info.value[0][1].name if isinstance(info, RObj) else None
        if cls == "compact_intseq":
            n, start, step = state.value
            v = RObj(13, (start + step * np.arange(int(n))).astype(np.int32))
        elif cls == "compact_realseq":
            n, start, step = state.value
            v = RObj(14, start + step * np.arange(int(n), dtype=np.float64))
        elif cls in ("wrap_integer", "wrap_real", "wrap_string", "wrap_logical"):
            v = state.value[0][1]
        elif cls == "deferred_string":
            arg = state.value[0][1]
            v = RObj(16, [str(x) for x in arg.value])
        else:
            raise ValueError(f"unsupported ALTREP class {cls}")
        if attr is not None:
            v.attr = self._attrs(attr)
        return v


def read_rda(path):
    """Return ``{name: RObj}`` for every object stored in an ``.rda`` file."""
    raw = gzip.open(path).read()
    if raw[:5] not in (b"RDX2\n", b"RDX3\n"):
        raise ValueError("not an XDR rda file")
    r = _Reader(raw)
    r.p = 5
    assert raw[r.p:r.p + 2] == b"X\n", "only XDR format supported"
    r.p += 2
    version = r.int()
    r.int()
    r.int()
    if version == 3:
        n = r.int()
        r.bytes_(n)
    top = r.item()
    out = {}
    for tag, car in top.value:
        out[tag.name] = car
    return out


# ---------------------------------------------------------------------------
# S4Vectors / IRanges / GenomicRanges decoding helpers
# ---------------------------------------------------------------------------

def rle_expand(rle):
    """S4Vectors::Rle -> numpy array of run values expanded."""
    vals = rle.a("values")
    lens = rle.a("lengths").value
    if vals.type == 16:
        v = np.array(vals.value, dtype=object)
    else:
        v = vals.value
    levels = vals.a("levels")
    if levels is not None:  # factor-valued Rle
        lv = np.array(levels.value, dtype=object)
        v = lv[np.asarray(v) - 1]
    return np.repeat(v, lens)


def granges_to_dict(gr):
    """GenomicRanges::GRanges -> plain arrays (1-based closed coordinates)."""
    rng = gr.a("ranges")
    start = rng.a("start").value.astype(np.int64)
    width = rng.a("width").value.astype(np.int64)
    names = rng.a("NAMES")
    seqnames = rle_expand(gr.a("seqnames"))
    strand = rle_expand(gr.a("strand"))
    si = gr.a("seqinfo")
    seqlevels = list(si.a("seqnames").value)
    seqlengths = si.a("seqlengths").value
    d = {
        "seqnames": np.array([str(s) for s in seqnames]),
        "start": start,
        "end": start + width - 1,
        "strand": np.array([str(s) for s in strand]),
        "seqlevels": np.array(seqlevels),
        "seqlengths": np.asarray(seqlengths, dtype=np.int64),
    }
    if names is not None:
        d["names"] = np.array([str(x) for x in names.value])
    return d


def dataframe_to_dict(df):
    cols = [str(x) for x in df.a("names").value]
    out = {}
    for name, col in zip(cols, df.value):
        if col.a("levels") is not None:
            lv = np.array(col.a("levels").value, dtype=object)
            out[name] = np.array([str(x) for x in lv[col.value - 1]])
        elif col.type == 16:
            out[name] = np.array([str(x) for x in col.value])
        else:
            out[name] = np.asarray(col.value)
    rn = df.a("row.names")
    if rn is not None and rn.type == 16:
        out["_rownames"] = np.array([str(x) for x in rn.value])
    return out
