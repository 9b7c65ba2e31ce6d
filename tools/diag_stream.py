"""Host-to-host paths of one C4 sample, repeated: the one-call streamed profile
(rcp_profile_reads), three samples in one call, and recoup()'s Rle path (readset, coverage_rle,
profile_rle), each `reps` times with the median and min.

    python tools/diag_stream.py [reps]      (RCP_TRACE=1: the pipelines' stderr lines)"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import synthetic  # noqa: E402
from recoup_amd.engine import (Bins, ReadSet, RowTable, coverage_rle_host, profile_reads,  # noqa: E402
                               profile_rle_arrays)

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 7
d = synthetic.c4(device="cuda:0")
reg = d["regions"]
rows = RowTable.from_ranges(reg["chrom"], reg["start"], reg["end"], reg["strand"])
bins = Bins([("whole", d["n_bins"])])
chrom, start, end, strand = d["reads"]
order = torch.argsort((chrom.to(torch.int64) << 32) | start.to(torch.int64))
sc = chrom[order]
rv, rl = torch.unique_consecutive(sc, return_counts=True)
w = (end[order] - start[order] + 1).to(torch.int32)
wv, wl = torch.unique_consecutive(w, return_counts=True)
host = [(rv.to(torch.int32).cpu().numpy(), rl.to(torch.int64).cpu().numpy()), start[order].cpu().numpy(),
        (wv.cpu().numpy(), wl.to(torch.int64).cpu().numpy()), strand[order].cpu().numpy()]
del order, sc, w
seqlen = d["seqlen"]
out = np.ones((bins.n_cols, rows.n_rows))
outs = [np.ones((bins.n_cols, rows.n_rows)) for _ in range(3)]
rle_out = np.ones((rows.n_rows, bins.n_cols), order="F")


ref = np.zeros((bins.n_cols, rows.n_rows))
profile_host_ref = __import__("recoup_amd.engine", fromlist=["profile_host"]).profile_host
profile_host_ref(ReadSet(*host, seqlen, device=0), rows, bins, ref, np.zeros(rows.n_rows, np.uint8))
bad = []


def check(name, m):
    m = np.asarray(m)
    if m.shape != ref.shape:
        m = m.T
    if not np.array_equal(m.view(np.int64), ref.view(np.int64)):
        diff = np.flatnonzero((m != ref).any(axis=0))
        bad.append(name)
        print(f"MISMATCH {name}: {diff.size} rows differ, first {diff[:8].tolist()} last {diff[-3:].tolist()}", flush=True)


def stats(name, xs):
    xs = sorted(xs)
    print(f"{name}: median {xs[len(xs) // 2]:.2f} ms, min {xs[0]:.2f}, all {[round(x, 1) for x in xs]}", flush=True)


one, three, rle, rle_ph, fresh = [], [], [], [], []
for k in range(max(3, reps // 2)):  # into a matrix never touched before, as R's allocMatrix gives it
    f = np.empty((bins.n_cols, rows.n_rows))
    a = time.perf_counter()
    profile_reads([host], seqlen, rows, bins, 0, [f])
    fresh.append((time.perf_counter() - a) * 1e3)
    check(f"fresh[{k}]", f)
    del f
for k in range(reps):
    torch.cuda.synchronize()
    a = time.perf_counter()
    profile_reads([host], seqlen, rows, bins, 0, [out])
    one.append((time.perf_counter() - a) * 1e3)
    check(f"one[{k}]", out)
    out[:] = 1.0
for k in range(max(3, reps // 2)):
    a = time.perf_counter()
    profile_reads([host] * 3, seqlen, rows, bins, 0, outs)
    three.append((time.perf_counter() - a) * 1e3 / 3)
    for j, o in enumerate(outs):
        check(f"three[{k}][{j}]", o)
        o[:] = 1.0
for k in range(max(3, reps // 2)):
    a = time.perf_counter()
    rs = ReadSet(*host, seqlen, device=0)
    b = time.perf_counter()
    run_off, values, lengths, valid = coverage_rle_host(rs, rows)
    c = time.perf_counter()
    profile_rle_arrays(run_off, lengths, values, (valid == 0).astype(np.uint8), bins, 0, rle_out)
    e = time.perf_counter()
    check(f"rle[{k}]", rle_out)
    rle_out[:] = 1.0
    del rs
    del run_off, values, lengths, valid
    rle.append((e - a) * 1e3)
    rle_ph.append(((b - a) * 1e3, (c - b) * 1e3, (e - c) * 1e3))
stats("one sample, one call", one)
stats("one sample, one call, fresh matrix", fresh)
stats("three samples, per sample", three)
stats("rle path", rle)
print("rle phases (readset, coverage_rle, profile_rle):", [tuple(round(x, 1) for x in p) for p in rle_ph])
print("mismatches:", bad)
