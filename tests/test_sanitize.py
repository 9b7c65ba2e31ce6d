"""ASan + UBSan build of the product's host code (rcp_host.cpp, rcp_bam.cpp) driven through
the C ABI on a corpus of truncated and corrupted BAM files (rcp_bam_read parses untrusted
input inside the caller's process -- an R session replacing readBam, R/ranges.R:111-132)
plus argument validation of every entry point.  CPU only: the device code is the regular
build's object and no kernel runs (host sanitizers)."""
import os
import struct
import subprocess
import zlib

import numpy as np
import pytest

from tests.test_bam import BAMS, _bgzf, _record

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SAN = os.path.join(HERE, "sanitize")
DRIVER = os.path.join(SAN, "build", "abi_driver")
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
           UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")


@pytest.fixture(scope="module")
def driver():
    if not all(os.path.exists(os.path.join(ROOT, "recoup_amd", "build", f)) for f in ("rcp_kernels.hip.o", "rcp_rle.hip.o")):
        from recoup_amd import build
        build.build(verbose=False)
    subprocess.check_call(["make", "-s", "-C", SAN], stdout=subprocess.DEVNULL)
    return DRIVER


def _run(driver, *args):
    p = subprocess.run([driver, *args], capture_output=True, text=True, env=ENV, timeout=300)
    out = p.stdout + p.stderr
    assert "AddressSanitizer" not in out and "runtime error" not in out and "LeakSanitizer" not in out, out[-4000:]
    assert p.returncode == 0, out[-4000:]
    return p.stdout


def test_abi_validation(driver):
    assert "abi ok" in _run(driver, "abi")


def _payload():
    hdr = b"BAM\1" + struct.pack("<i", 3) + b"@H\n" + struct.pack("<i", 2)
    for name, ln in (("chrA", 5000), ("chrB", 800)):
        hdr += struct.pack("<i", len(name) + 1) + name.encode() + b"\0" + struct.pack("<i", ln)
    recs = [_record(i % 2, (37 * i) % 700, (0, 16, 4)[i % 3], [(30, "M"), (50, "N"), (20, "M")], b"q%d" % i)
            for i in range(60)]
    return hdr, b"".join(recs)


def _block(raw_deflate, isize, crc=0, xlen_extra=b"", bsize=None):
    """One gzip member with a hand-set BSIZE / extra field."""
    extra = struct.pack("<BBHH", 66, 67, 2, 0) + xlen_extra
    blen = 12 + len(extra) + len(raw_deflate) + 8
    extra = struct.pack("<BBHH", 66, 67, 2, (blen - 1) if bsize is None else bsize) + xlen_extra
    return (struct.pack("<BBBBIBBH", 31, 139, 8, 4, 0, 0, 255, len(extra)) + extra + raw_deflate +
            struct.pack("<II", crc, isize))


def _deflate(b):
    c = zlib.compressobj(6, zlib.DEFLATED, -15)
    return c.compress(b) + c.flush()


def corpus(tmp):
    hdr, recs = _payload()
    good = _bgzf(hdr + recs, block=700)
    files = {"good": good}
    # truncations at many offsets (inside block headers, extra fields, deflate data, trailers)
    for k in sorted(set(np.linspace(1, len(good) - 1, 80).astype(int).tolist() + list(range(1, 40)))):
        files[f"trunc{k}"] = good[:k]
    # BGZF framing
    files["xlen_huge"] = struct.pack("<BBBBIBBH", 31, 139, 8, 4, 0, 0, 255, 65535) + b"BC\x02\x00\x10\x00" + b"\0" * 12
    files["slen_beyond"] = struct.pack("<BBBBIBBH", 31, 139, 8, 4, 0, 0, 255, 6) + b"BC\xff\x7f\x10\x00" + b"\0" * 40
    files["no_bsize"] = struct.pack("<BBBBIBBH", 31, 139, 8, 4, 0, 0, 255, 6) + b"XY\x02\x00\x10\x00" + b"\0" * 40
    files["bsize_small"] = _block(_deflate(hdr), len(hdr), bsize=10)
    files["bsize_past_eof"] = _block(_deflate(hdr), len(hdr), bsize=60000)
    files["isize_huge"] = _block(_deflate(hdr), 1 << 30)
    files["isize_short"] = _block(_deflate(hdr), 3)
    files["isize_long"] = _block(_deflate(hdr), len(hdr) + 100)
    files["deflate_garbage"] = _block(b"\xff" * 50, 100)
    files["two_subfields"] = _block(_deflate(hdr), len(hdr), xlen_extra=b"ZZ\x03\x00abc")
    files["not_gzip"] = b"BAM\1" * 40
    # BAM payload (valid BGZF around it)
    bad = {
        "l_text_huge": b"BAM\1" + struct.pack("<i", 2 ** 31 - 1) + hdr[8:],
        "l_text_neg": b"BAM\1" + struct.pack("<i", -5) + hdr[8:],
        "n_ref_huge": hdr[:11] + struct.pack("<i", 2 ** 31 - 1) + hdr[15:],
        "n_ref_neg": hdr[:11] + struct.pack("<i", -3) + hdr[15:] + recs,
        "l_name_zero": hdr[:15] + struct.pack("<i", 0) + hdr[19:] + recs,
        "l_name_huge": hdr[:15] + struct.pack("<i", 2 ** 30) + hdr[19:] + recs,
        "bad_magic": b"BAX\1" + hdr[4:] + recs,
        "block_size_small": hdr + struct.pack("<i", 8) + recs[4:],
        "block_size_huge": hdr + struct.pack("<i", 2 ** 31 - 1) + recs[4:],
        "block_size_neg": hdr + struct.pack("<i", -40) + recs[4:],
    }
    r0 = bytearray(recs)
    r0[4 + 12:4 + 14] = struct.pack("<H", 65535)  # n_cigar beyond the record
    bad["n_cigar_beyond"] = hdr + bytes(r0)
    r1 = bytearray(recs)
    r1[4 + 8] = 255  # l_read_name beyond the record
    bad["read_name_beyond"] = hdr + bytes(r1)
    r2 = bytearray(recs)
    r2[4:8] = struct.pack("<i", 99)  # reference index out of range
    bad["ref_out_of_range"] = hdr + bytes(r2)
    r3 = bytearray(recs)
    r3[4 + 4:4 + 8] = struct.pack("<i", 2 ** 31 - 10)  # position near INT32_MAX
    bad["pos_huge"] = hdr + bytes(r3)
    for k, v in bad.items():
        files[k] = _bgzf(v, block=500)
    # seeded byte flips in the decompressed stream
    rng = np.random.default_rng(11)
    raw = bytearray(hdr + recs)
    for i in range(60):
        x = bytearray(raw)
        for pos in rng.integers(0, len(x), int(rng.integers(1, 6))):
            x[int(pos)] = int(rng.integers(0, 256))
        files[f"flip{i}"] = _bgzf(bytes(x), block=int(rng.integers(100, 2000)))
    paths = []
    for k, v in files.items():
        p = os.path.join(tmp, k + ".bam")
        with open(p, "wb") as f:
            f.write(v)
        paths.append(p)
    return paths


def test_corrupt_bam_corpus(driver, tmp_path):
    paths = corpus(str(tmp_path))
    out = _run(driver, "bam", *paths, *BAMS)
    rc = {}
    for line in out.splitlines():
        path, action, code, n = line.rsplit(" ", 3)
        rc.setdefault(os.path.basename(path), set()).add(int(code))
    assert len(rc) == len(paths) + len(BAMS)
    assert rc["good.bam"] == {0}
    for b in BAMS:
        assert rc[os.path.basename(b)] == {0}
    for k in ("xlen_huge", "slen_beyond", "no_bsize", "bsize_small", "bsize_past_eof", "isize_huge",
              "isize_short", "isize_long", "deflate_garbage", "not_gzip", "l_text_huge", "n_ref_huge",
              "l_name_zero", "l_name_huge", "bad_magic", "block_size_small", "block_size_huge", "block_size_neg",
              "n_cigar_beyond", "read_name_beyond"):
        assert rc[k + ".bam"] <= {-1, -3, -5} and 0 not in rc[k + ".bam"], (k, rc[k + ".bam"])
    assert rc["two_subfields.bam"] == {0}  # extra subfields before/after BC are legal
