"""Benchmark of the recoup coverage -> profile hot path on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c4|c2|c5]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

A step is one pass of the hot path -- calcCoverage + profileMatrix fused: locate kernel,
LDS pileup-bin kernel, interpolation kernel -- over one synthetic C4 sample
(200k ChIP peak summits +-1 kb, 1000 bins, 200M reads) with the reads, region tables and
output matrix already resident in HBM.  Each rank holds its own C4 partition (regions and
reads are independent objects: weak scaling, no collective on the data path).

Prints ONE JSON line (rank 0): value = region-bins/s over all ranks, plus
  roofline      the pileup kernel's algorithmic bytes / its HIP-event-timed duration
  cpu_baseline  the CPU oracle (test infrastructure, `oracle/`) on a bounded sample, timed here
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


# plan.info["pileup_kernel"] -> kernel name (as rocprofv3 lists it)
PILEUP_KERNELS = {0: "rcp_pileup_kernel", 1: "rcp_pileup_lean_kernel", 2: "rcp_pileup_lean_kernel (general bins)"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c4", choices=["c4", "c2", "c3", "c5"])
    ap.add_argument("--seed", type=int, default=20261015)
    ap.add_argument("--reads", type=int, default=None, help="override read count (smaller runs)")
    ap.add_argument("--regions", type=int, default=None, help="override region count")
    ap.add_argument("--cpu-regions", type=int, default=200000, help="CPU baseline sample (regions)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline: repeat the sample this long")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the one-off host-to-host timing")
    ap.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "traffic_c4.json"),
                    help="PMC traffic summary (from tools/pmc_traffic.py) to attach to the roofline")
    return ap.parse_args()


def log(*a):
    print(*a, file=sys.stderr, flush=True)


WORKLOADS = {
    "c4": "C4: 200k ChIP peak summits +-1 kb, 1000 bins (2 bp), 200M reads (180 bp)",
    "c2": "C2: 10k TSS +-2 kb, 200 bins, 10M reads (180 bp)",
    "c3": "C3: coverageRnaRef, 25k genes (exon lists + 2 kb flanks), 50 + 500 + 50 bins, 50M read pairs "
          "(100 bp mates, junction reads split)",
    "c5": "C5: 25k regions x 4000 bp per base, 500M reads (50 bp)",
}


def workload(args, dev, rank):
    """(data, RowTable, Bins, total read-segment overlaps) of the chosen BASELINE config."""
    import synthetic
    from recoup_amd.engine import Bins, RowTable
    seed = args.seed + 7919 * rank
    if args.config == "c3":
        kw = {}
        if args.reads:
            kw["n_pairs"] = args.reads // 2
        if args.regions:
            kw["n_genes"] = args.regions
        d = synthetic.c3(device=dev, seed=seed, **kw)
        rows = synthetic.rna_rows(d)
        bins = Bins([("upstream", d["flank_bins"]), ("center", d["region_bins"]), ("downstream", d["flank_bins"])],
                    flank=d["flank"])
        ovl = synthetic.n_overlaps_segments(d["reads"], rows.chrom, rows.start, rows.end, device=dev).sum()
        return d, rows, bins, ovl
    kw = {}
    if args.reads:
        kw["n_reads"] = args.reads
    if args.regions:
        kw["n_regions"] = args.regions
    d = getattr(synthetic, args.config)(device=dev, seed=seed, **kw)
    reg = d["regions"]
    rows = RowTable.from_ranges(reg["chrom"], reg["start"], reg["end"], reg["strand"])
    bins = Bins([("whole", d["n_bins"])]) if d["n_bins"] > 0 else Bins([("whole", 0, sum(d["flank"]))])
    ovl = synthetic.n_overlaps(d["reads"], reg, d["width"], device=dev).sum()
    return d, rows, bins, ovl


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = world > 1
    # rehearsal of the N > 1 path on fewer GPUs: RCP_DIST_BACKEND=gloo RCP_SHARE_GPU=1 puts
    # several ranks on one device and the barrier / max-reduction on the host
    backend = os.environ.get("RCP_DIST_BACKEND", "nccl")
    if os.environ.get("RCP_SHARE_GPU") == "1":
        local = local % torch.cuda.device_count()
    if dist:
        import torch.distributed as tdist
        torch.cuda.set_device(local)
        if backend == "nccl":
            tdist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
        else:
            tdist.init_process_group(backend)
    dev = f"cuda:{local}"
    torch.cuda.set_device(local)

    from recoup_amd.engine import Plan, ReadSet

    t0 = time.time()
    data, rows, bins, ovl_rows = workload(args, dev, rank)
    reads = data["reads"]
    R = rows.n_rows
    n_reads = int(reads[1].numel())
    torch.cuda.synchronize()
    log(f"[rank {rank}] data {args.config}: {n_reads} reads, {R} rows in {time.time() - t0:.1f}s")

    t1 = time.time()
    rs = ReadSet(*reads, data["seqlen"], device=local)
    tp = time.time()
    plan = Plan(rs, rows, bins)
    plan_s = time.time() - tp
    B = plan.n_cols
    out = plan.empty_output()
    valid = torch.empty(R, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    log(f"[rank {rank}] readset + plan in {time.time() - t1:.1f}s (plan {plan_s * 1e3:.1f} ms), info {plan.info}")

    # ---- warmup + correctness gate
    for _ in range(args.warmup):
        plan.execute(out, valid)
    plan.status()

    # ---- timed region: exactly K steps between barrier + synchronize
    if dist:
        tdist.barrier()
    torch.cuda.synchronize()
    ts = time.perf_counter()
    for _ in range(args.steps):
        plan.execute(out, valid)
    torch.cuda.synchronize()
    if dist:
        tdist.barrier()
    elapsed = time.perf_counter() - ts
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        elapsed = float(t.item())
    plan.status()

    # ---- per-kernel durations with HIP events on the launch stream
    stream = torch.cuda.current_stream()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    kt = np.zeros(3)
    for _ in range(args.steps):
        ev[0].record(stream)
        plan.execute_stages(1, out, valid)
        ev[1].record(stream)
        plan.execute_stages(2, out)
        ev[2].record(stream)
        plan.execute_stages(4, out)
        ev[3].record(stream)
        torch.cuda.synchronize()
        kt += [ev[0].elapsed_time(ev[1]), ev[1].elapsed_time(ev[2]), ev[2].elapsed_time(ev[3])]
    kt /= args.steps  # ms per launch
    plan.status()

    units = R * B  # region-bins per step per rank (1 sample)
    value = world * units * args.steps / elapsed
    ovl = int(ovl_rows)
    # 8 B per overlapping (read, segment) + 16 B per region + 8 B per further segment
    # of a multi-range row + the f64 output written once
    n_seg = len(rows.start)
    bytes_pileup = 8 * ovl + 16 * R + 8 * (n_seg - R) + 8 * R * B
    achieved = bytes_pileup / (kt[1] * 1e-3) / 1e9
    traffic = None
    if os.path.exists(args.traffic):
        try:
            tr = json.load(open(args.traffic))
            if tr.get("config") == args.config and tr.get("regions") == R and tr.get("reads") == n_reads:
                traffic = tr.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    # ---- end to end once (not `value`): what a host caller (the R shim's rcp_profile) pays --
    # host read arrays -> H2D + device sort (readset), plan, one pass, D2H of the matrix
    e2e = None
    if not args.no_e2e:
        e2e = end_to_end(data, rows, bins, local, R * B)
        if dist:
            t = torch.tensor([e2e["ms"]], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
            tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
            e2e["ms"] = float(t.item())
            e2e["region_bins_per_s"] = world * R * B / (e2e["ms"] * 1e-3)

    # ---- CPU baseline (rank 0, N = 1): the oracle on a bounded sample of the same workload
    cpu = None
    parity = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu, parity = cpu_baseline(args, data, rows, bins, out, valid, B)

    if rank == 0:
        res = {
            "metric": "region-bins/sec (profileMatrix)",
            "value": value,
            "unit": "region-bins/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic",
            "config": {
                "workload": WORKLOADS[args.config],
                "regions_per_gpu": R, "bins": B, "reads_per_gpu": n_reads, "samples": 1,
                "parallelism": f"region-sharded x{world} (one partition per GPU, no data-path collective)",
            },
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBPS, "traffic": traffic,
                         "kernel": PILEUP_KERNELS[plan.info["pileup_kernel"]],
                         "algorithmic_bytes_per_launch": bytes_pileup,
                         "kernel_ms": kt[1]},
            "cpu_baseline": cpu,
            "e2e": e2e,
            "kernel_ms": {"locate": kt[0], "pileup": kt[1], "interp": kt[2]},
            "n_overlaps": ovl,
            "plan_ms": plan_s * 1e3,
            "parity_sample": parity,
        }
        print(json.dumps(res), flush=True)
    if dist:
        tdist.destroy_process_group()


def end_to_end(data, rows, bins, local, units):
    """One host-to-host pass, timed in phases: pageable host read arrays (as R holds them) ->
    ReadSet (H2D + device radix sort + stream index) -> Plan -> execute -> D2H of the R
    column-major matrix into pageable host memory.  Reported beside `value`, never as it."""
    from recoup_amd.engine import Plan, ReadSet
    host = [x.cpu().numpy() for x in data["reads"]]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    rs = ReadSet(*host, data["seqlen"], device=local)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    plan = Plan(rs, rows, bins)
    t2 = time.perf_counter()
    out = plan.empty_output()
    plan.execute(out)
    torch.cuda.synchronize()
    t3 = time.perf_counter()
    mat = out.cpu()
    t4 = time.perf_counter()
    plan.status()
    del plan, rs, out, mat
    ms = (t4 - t0) * 1e3
    return {"ms": ms, "region_bins_per_s": units / (ms * 1e-3),
            "phases_ms": {"readset_h2d_sort": (t1 - t0) * 1e3, "plan": (t2 - t1) * 1e3,
                          "execute": (t3 - t2) * 1e3, "d2h_matrix": (t4 - t3) * 1e3},
            "note": "one pass from pageable host arrays to a host matrix; includes PCIe both ways"}


def cpu_baseline(args, data, rows, bins, out, valid, B):
    """The oracle (C restatement of the reference's per-region dataflow, multithreaded over
    regions like cmclapply with rc = NULL) on the first --cpu-regions rows, repeated for about
    --cpu-seconds; multi-range rows (C3) go through the oracle's per-group coverage + splitVector."""
    from oracle import oracle as o
    R = rows.n_rows
    m = min(args.cpu_regions, R)
    chrom, start, end, strand = data["reads"]
    keep = np.unique(rows.chrom[:rows.seg_off[m]])
    sel = torch.isin(chrom, torch.as_tensor(keep, device=chrom.device, dtype=chrom.dtype))
    # hand the oracle its reads in (chrom, start) order so its own index skips the sort
    c, s, e, st = chrom[sel], start[sel], end[sel], strand[sel]
    key = (c.to(torch.int64) << 42) + (s.to(torch.int64) << 10) + (e - s).to(torch.int64).clamp(0, 1023)
    order = torch.argsort(key)
    c, s, e, st = (x[order].cpu().numpy() for x in (c, s, e, st))
    ix = o.Index(c, s, e, st, data["seqlen"])
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:
        cores = os.cpu_count() or 1
    threads = max(1, min(16, cores))
    single = bool(np.all(np.diff(rows.seg_off[:m + 1]) == 1)) and len(bins.parts) == 1
    if single:
        mask = o.Mask.from_ranges(rows.chrom[:m], rows.start[:m], rows.end[:m], rows.strand[:m])
        nb = int(bins.n_bins[0])

        def run():
            if nb > 0:
                return o.profile_part(ix, mask, nb, nthreads=threads)
            return o.profile_part(ix, mask, 0, ncol=B, nthreads=threads)
    else:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_rows
        from recoup_amd.engine import RowTable
        sub = RowTable(rows.seg_off[:m + 1], rows.chrom[:rows.seg_off[m]], rows.start[:rows.seg_off[m]],
                       rows.end[:rows.seg_off[m]], rows.strand[:rows.seg_off[m]],
                       seg_group=None if rows.seg_group is None else rows.seg_group[:rows.seg_off[m]],
                       group_is_list=rows.group_is_list, ignore_strand=rows.ignore_strand)
        threads = 1

        def run():
            return oracle_rows.profile(oracle_rows.row_coverage(ix, sub), bins)
    # repeat the sample until about args.cpu_seconds of wall time (a single pass over C4 takes
    # well under a second on a many-core host) and report the mean pass
    reps = 0
    t = time.perf_counter()
    while True:
        ref, rvalid = run()
        reps += 1
        if time.perf_counter() - t >= args.cpu_seconds:
            break
    dt = (time.perf_counter() - t) / reps
    gpu = out.cpu().numpy().T[:m]
    gv = valid.cpu().numpy()[:m].astype(bool)
    # NaN where the reference's neighborhood fill averages four NAs (mean(na.rm = TRUE) of nothing)
    parity = bool(np.array_equal(gv, np.asarray(rvalid).astype(bool)) and
                  np.allclose(gpu, ref, rtol=1e-9, atol=1e-12, equal_nan=True))
    cpu = {"value": m * B / dt, "unit": "region-bins/s", "cores": threads, "kind": "port",
           "sample": f"first {m} of {R} rows (all their reads), {B} columns; oracle/ C restatement"
                     f"{', %d threads over regions' % threads if single else ' (per-group coverage, Python splitVector)'}; "
                     f"mean of {reps} passes, {dt:.3f} s/pass"}
    return cpu, parity


if __name__ == "__main__":
    main()
