"""BAM ingest (readBam, R/ranges.R:111-146) through librecoup_amd.so on the host.

Checked against an independent pure-Python restatement (gzip + struct) on
  * the reference's own BAM fixtures (inst/extdata/*_50kr.bam, copied to tests/golden/bam), and
  * synthetic BAMs written here with every CIGAR operation, unmapped records, reverse strands,
    alignments running past the sequence end, several references and many BGZF blocks.
R is absent, so agreement with readGAlignments / grglist / trim is "parity unpinned" beyond
the SAM specification these restate."""
import gzip
import os
import struct
import zlib

import numpy as np
import pytest

import recoup_amd as ra

HERE = os.path.dirname(os.path.abspath(__file__))
BAMS = [os.path.join(HERE, "golden", "bam", f) for f in ("WT_H4K20me1_50kr.bam", "Set8KO_H4K20me1_50kr.bam")]
OPS = "MIDNSHP=X"


# ------------------------------------------------------------------ restatement (oracle)
def py_read_bam(path, action="keep", q=0.75):
    d = gzip.open(path).read()
    assert d[:4] == b"BAM\1"
    o = 8 + struct.unpack("<i", d[4:8])[0]
    n_ref = struct.unpack("<i", d[o:o + 4])[0]
    o += 4
    names, lens = [], []
    for _ in range(n_ref):
        ln = struct.unpack("<i", d[o:o + 4])[0]
        names.append(d[o + 4:o + 3 + ln].decode())
        lens.append(struct.unpack("<i", d[o + 4 + ln:o + 8 + ln])[0])
        o += 8 + ln
    rows = []
    while o < len(d):
        bs = struct.unpack("<i", d[o:o + 4])[0]
        ref, pos, lrn, _mapq, _bin, ncig, flag = struct.unpack("<iiBBHHH", d[o + 4:o + 20])
        cig = struct.unpack(f"<{ncig}I", d[o + 36 + lrn:o + 36 + lrn + 4 * ncig])
        o += 4 + bs
        if flag & 4 or ref < 0:
            continue
        st = 1 if flag & 16 else 0
        sl = lens[ref]
        trim = lambda a, b: (max(a, 1), max(min(b, sl), max(a, 1) - 1))  # noqa: E731
        x = pos + 1
        if action == "split":
            b0 = x
            got = False
            for v in cig:
                op, ln = OPS[v & 15], v >> 4
                if op == "N":
                    if x > b0:
                        rows.append((ref, *trim(b0, x - 1), st))
                        got = True
                    x += ln
                    b0 = x
                elif op in "MD=X":
                    x += ln
            if x > b0 or not got:
                rows.append((ref, *trim(b0, x - 1), st))
        else:
            w = sum(v >> 4 for v in cig if OPS[v & 15] in "MDN=X")
            rows.append((ref, *trim(pos + 1, pos + w), st))
    a = np.array(rows, dtype=np.int64).reshape(-1, 4)
    if action == "remove" and len(a):
        w = a[:, 2] - a[:, 1] + 1
        a = a[w <= np.quantile(w, q)]
    return names, lens, a


# ------------------------------------------------------------------ synthetic BAM writer
def _bgzf(data, block=4000):
    out = bytearray()
    for i in range(0, len(data), block):
        chunk = data[i:i + block]
        c = zlib.compressobj(6, zlib.DEFLATED, -15)
        comp = c.compress(chunk) + c.flush()
        out += struct.pack("<BBBBIBBHBBHH", 31, 139, 8, 4, 0, 0, 255, 6, 66, 67, 2, len(comp) + 25)
        out += comp + struct.pack("<II", zlib.crc32(chunk) & 0xFFFFFFFF, len(chunk))
    out += bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000")  # EOF block
    return bytes(out)


def _record(ref, pos, flag, cigar, name=b"r"):
    ops = [(int(n), OPS.index(op)) for n, op in cigar]
    l_seq = sum(n for n, op in ops if OPS[op] in "MIS=X")
    core = struct.pack("<iiBBHHHiiii", ref, pos, len(name) + 1, 60, 0, len(ops), flag, l_seq, -1, -1, 0)
    body = name + b"\0" + b"".join(struct.pack("<I", (n << 4) | op) for n, op in ops)
    body += b"\x11" * ((l_seq + 1) // 2) + b"\xff" * l_seq
    return struct.pack("<i", len(core) + len(body)) + core + body


def write_bam(path, refs, recs):
    hdr = b"BAM\1" + struct.pack("<i", 0) + struct.pack("<i", len(refs))
    for name, ln in refs:
        hdr += struct.pack("<i", len(name) + 1) + name.encode() + b"\0" + struct.pack("<i", ln)
    data = hdr + b"".join(_record(*r) for r in recs)
    with open(path, "wb") as f:
        f.write(_bgzf(data))


@pytest.fixture(scope="module")
def synthetic_bam(tmp_path_factory):
    rng = np.random.default_rng(3)
    refs = [("chrA", 50000), ("chrB", 8000), ("chrC", 300)]
    recs = []
    shapes = [[(100, "M")], [(30, "S"), (70, "M")], [(40, "M"), (500, "N"), (60, "M")],
              [(20, "M"), (5, "D"), (20, "M"), (2, "I"), (30, "M")], [(10, "H"), (50, "=")],
              [(25, "M"), (100, "N"), (25, "X"), (1000, "N"), (30, "M")], [(50, "M"), (10, "N")]]
    for i in range(3000):
        ref = int(rng.integers(0, 3))
        pos = int(rng.integers(0, refs[ref][1] - 50))  # some run past the end (trim)
        flag = int(rng.choice([0, 16, 4, 0, 16, 1024, 256]))
        recs.append((ref if flag != 4 or i % 2 else -1, pos, flag, shapes[i % len(shapes)], b"q%d" % i))
    path = str(tmp_path_factory.mktemp("bam") / "synthetic.bam")
    write_bam(path, refs, recs)
    return path


def _check(path, action, q=0.75):
    names, lens, exp = py_read_bam(path, action, q)
    g = ra.readBam(path, spliceAction=action, spliceRemoveQ=q, threads=4)
    assert g.seqlevels == names
    np.testing.assert_array_equal(g.seqlengths, lens)
    got = np.stack([g.seqcodes, g.start, g.end, g.strand], axis=1).astype(np.int64)
    np.testing.assert_array_equal(got, exp)
    return g


@pytest.mark.parametrize("path", BAMS)
def test_reference_fixture_bams(path):
    g = _check(path, "keep")
    assert len(g) == 50000 and g.seqlevels == ["chr12"] and set(g.width) == {180}
    _check(path, "split")
    _check(path, "remove")


@pytest.mark.parametrize("action", ["keep", "split", "remove"])
def test_synthetic_bam(synthetic_bam, action):
    g = _check(synthetic_bam, action, q=0.6)
    assert len(g.seqlevels) == 3


def test_split_makes_blocks(synthetic_bam):
    keep = ra.readBam(synthetic_bam, "keep")
    split = ra.readBam(synthetic_bam, "split")
    assert len(split) > len(keep)  # N-skips become separate ranges
    assert split.width.sum() < keep.width.sum()


def test_bad_files(tmp_path):
    p = tmp_path / "x.bam"
    p.write_bytes(b"not a bam at all" * 4)
    with pytest.raises(ra.RcpError):
        ra.readBam(str(p))
    with pytest.raises(ra.RcpError):
        ra.readBam(str(tmp_path / "missing.bam"))
    good = open(BAMS[0], "rb").read()
    p.write_bytes(good[:len(good) // 2])
    with pytest.raises(ra.RcpError):
        ra.readBam(str(p))
