"""Benchmark of the recoup coverage -> profile hot path on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c4|c2|c3|c5]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

`--gpus N > 1` without a torch.distributed environment (WORLD_SIZE unset) starts the N ranks
itself: torch.distributed.run as a CHILD process (this process never touches a GPU; it exits
with the launcher's status), after checking that N devices are visible (RCP_SHARE_GPU=1: a
rehearsal of N ranks on fewer GPUs, over gloo).  Under a launcher, --gpus must equal WORLD_SIZE.

A step is one pass of the hot path -- calcCoverage + profileMatrix fused: locate,
heavy-slice, pileup-bin and interpolation kernels -- over one synthetic workload (default
C4: 200k ChIP peak summits +-1 kb, 1000 bins, 200M reads) with the reads, region tables and
output matrix already resident in HBM.  With N ranks the ONE workload is region-sharded
(BASELINE config 4 "region-sharded across 8xMI355X"): regions sorted by
(chromosome, start) are cut into N contiguous shards balanced by overlapping reads, each rank
indexes only the reads its shard touches and computes its rows; no collective on the data
path (strong scaling: value = all regions x bins / the slowest rank's time).  The optional
reassembly of the R x B matrix (one RCCL all_gather over xGMI) is timed separately
(`gather`), never inside `value`.

Prints ONE JSON line (rank 0): value = region-bins/s of the whole job, plus
  roofline      the pileup kernel's algorithmic bytes / its HIP-event-timed duration (rank 0's
                shard), PMC traffic of the same kernel when profiles/ holds it, and the
                whole-step fraction
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
PILEUP_KERNELS = {0: "rcp_pileup_kernel", 1: "rcp_pileup_lean_kernel", 2: "rcp_pileup_lean_kernel (general bins)",
                  3: "rcp_pileup_rows_kernel", 4: "rcp_pileup_bins_kernel"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (ranks, one per GPU); default WORLD_SIZE under a launcher, else 1")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c4", choices=["c4", "c2", "c3", "c5"])
    ap.add_argument("--seed", type=int, default=20261015)
    ap.add_argument("--reads", type=int, default=None, help="override read count (smaller runs)")
    ap.add_argument("--regions", type=int, default=None, help="override region count")
    ap.add_argument("--cpu-regions", type=int, default=200000, help="CPU baseline sample (regions)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline: repeat the sample this long")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--sim-shard", default=None, metavar="K/N",
                    help="one GPU runs exactly rank K's shard of an N-way split (strong-scaling rehearsal)")
    ap.add_argument("--verify-gather", action="store_true",
                    help="N > 1: rank 0 also runs the whole workload alone and checks the gathered matrix bit for bit")
    ap.add_argument("--no-e2e", action="store_true", help="skip the one-off host-to-host timing")
    ap.add_argument("--kernel", default="auto", help="pileup kernel of the timed plans (A/B; default auto)")
    ap.add_argument("--inflight", default="auto", choices=["auto", "1", "2", "3", "4"],
                    help="samples in flight: D DISTINCT samples (independent read sets over the same region "
                         "table, as profileMatrix loops over a recoup input list) on D HIP streams, step k "
                         "= one complete pass of sample k %% D; auto (default): the fastest of 1, 2, 3, 4, "
                         "timed on every rank (max over ranks) so all ranks run the same D.  The "
                         "one-sample pass time is always reported beside it (single_pass_ms)")
    ap.add_argument("--traffic", default=None,
                    help="PMC traffic summary (tools/pmc_traffic.py); default profiles/traffic_<config>.json")
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


def workload(args, dev, sample=0):
    """(data, RowTable, Bins, per-row overlapping read-segment pairs) of the chosen BASELINE
    config.  Every rank generates the SAME data (one seed, Philox on the device); ``sample`` k
    > 0 is another sample's reads over the same regions."""
    import synthetic
    from recoup_amd.engine import Bins, RowTable
    seed = args.seed
    if args.config == "c3":
        kw = {"sample": sample}
        if args.reads:
            kw["n_pairs"] = args.reads // 2
        if args.regions:
            kw["n_genes"] = args.regions
        d = synthetic.c3(device=dev, seed=seed, **kw)
        rows = synthetic.rna_rows(d)
        bins = Bins([("upstream", d["flank_bins"]), ("center", d["region_bins"]), ("downstream", d["flank_bins"])],
                    flank=d["flank"])
        seg = synthetic.n_overlaps_segments(d["reads"], rows.chrom, rows.start, rows.end, device=dev)
        ovl = np.add.reduceat(seg, rows.seg_off[:-1]) if len(seg) else np.zeros(rows.n_rows, np.int64)
        return d, rows, bins, ovl.astype(np.int64)
    kw = {"sample": sample}
    if args.reads:
        kw["n_reads"] = args.reads
    if args.regions:
        kw["n_regions"] = args.regions
    d = getattr(synthetic, args.config)(device=dev, seed=seed, **kw)
    reg = d["regions"]
    rows = RowTable.from_ranges(reg["chrom"], reg["start"], reg["end"], reg["strand"])
    bins = Bins([("whole", d["n_bins"])]) if d["n_bins"] > 0 else Bins([("whole", 0, sum(d["flank"]))])
    ovl = synthetic.n_overlaps(d["reads"], reg, d["width"], device=dev).astype(np.int64)
    return d, rows, bins, ovl


def gpu_sleep(seconds):
    """Keep the current stream busy for about `seconds` (torch's spin kernel; a no-op where it is
    missing): the host enqueues the following launches meanwhile."""
    try:
        torch.cuda._sleep(int(seconds * 2.4e9))  # (cycles at ~2.4 GHz)
    except (AttributeError, RuntimeError):
        pass


def shard_of(rows, ovl, world, rank, per_region=64.0):
    """Rows [lo, hi) of this rank: contiguous in (chromosome, start) order (the synthetic
    region tables are sorted that way), balanced by overlapping reads + a per-region constant
    (recoup_amd.shard.balance)."""
    from recoup_amd.shard import balance
    cuts = balance(np.asarray(ovl, np.float64) + per_region, world)
    return int(cuts[rank]), int(cuts[rank + 1]), cuts


def subset_rows(rows, lo, hi):
    from recoup_amd.engine import RowTable
    j0, j1 = int(rows.seg_off[lo]), int(rows.seg_off[hi])
    sl = slice(j0, j1)
    return RowTable(rows.seg_off[lo:hi + 1] - j0, rows.chrom[sl], rows.start[sl], rows.end[sl], rows.strand[sl],
                    seg_group=None if rows.seg_group is None else rows.seg_group[sl],
                    group_is_list=rows.group_is_list, ignore_strand=rows.ignore_strand)


def reads_for_rows(reads, rows, n_chrom):
    """The reads a shard can touch, selected on the device: per chromosome, those overlapping
    [min segment start, max segment end] of the shard's rows.  A row's coverage depends only
    on the reads it hits (with NA seqlengths its Rle length is their max end,
    R/coverage.R:201), so the shard's rows are unchanged (recoup_amd.shard.reads_for)."""
    chrom, start, end, strand = reads
    dev = start.device
    lo = torch.full((n_chrom,), 2 ** 31 - 1, dtype=torch.int64, device=dev)
    hi = torch.full((n_chrom,), -(2 ** 31), dtype=torch.int64, device=dev)
    c = torch.as_tensor(rows.chrom, dtype=torch.int64, device=dev)
    if c.numel():
        lo.scatter_reduce_(0, c, torch.as_tensor(rows.start, dtype=torch.int64, device=dev), "amin")
        hi.scatter_reduce_(0, c, torch.as_tensor(rows.end, dtype=torch.int64, device=dev), "amax")
    ci = chrom.to(torch.int64)
    keep = (end.to(torch.int64) >= lo[ci]) & (start.to(torch.int64) <= hi[ci])
    return tuple(x[keep].contiguous() for x in (chrom, start, end, strand))


def host_cores():
    """CPU threads this process may use: the affinity mask, capped by a cgroup CPU quota
    (cpu.max) when one is set.  Returns (threads, basis string)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    n, basis = aff, f"sched_getaffinity {aff}"
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) // int(per)))
            basis += f", cgroup cpu.max {quota}"
            n = min(n, quota)
    except (OSError, ValueError):
        pass
    return n, basis


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def load_traffic(path, args, kernel, R, n_reads, world):
    """PMC traffic per launch of THIS kernel on THIS workload (tools/pmc_traffic.py), else None."""
    if not path or not os.path.exists(path) or world != 1:
        return None
    try:
        tr = json.load(open(path))
    except (OSError, ValueError):
        return None
    if (tr.get("config") == args.config and tr.get("regions") == R and tr.get("reads") == n_reads
            and tr.get("kernel") == kernel):
        return tr.get("hbm_bytes_per_launch")
    return None


class Refused(SystemExit):
    """A bench configuration that cannot run as asked (exit status 2, message on stderr)."""

    def __init__(self, msg):
        log(f"bench.py: {msg}")
        super().__init__(2)


def free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_plan(args, env, n_visible, argv, port=None):
    """How this invocation runs: (world, None) to run here as one rank of `world`, or (N, cmd)
    to start N ranks as a child torch.distributed.run.  `n_visible` = torch.cuda.device_count()
    (on this image that count does not initialise the GPU, so the launcher process never does).
    Refuses (exit status 2) when N GPUs are asked for and fewer are visible -- unless
    RCP_SHARE_GPU=1 (several ranks per device: a rehearsal) -- or when --gpus disagrees with the
    launcher's WORLD_SIZE."""
    share = env.get("RCP_SHARE_GPU") == "1"
    if env.get("WORLD_SIZE") is not None:
        world = int(env["WORLD_SIZE"])
        if args.gpus is not None and args.gpus != world:
            raise Refused(f"--gpus {args.gpus} but the launcher started WORLD_SIZE = {world} ranks")
        if not share and n_visible < world:
            raise Refused(f"{world} ranks but {n_visible} visible GPU(s) (RCP_SHARE_GPU=1 to share them)")
        return world, None
    n = 1 if args.gpus is None else args.gpus
    if n < 1:
        raise Refused(f"--gpus {n}")
    if not share and n_visible < n:
        raise Refused(f"--gpus {n} but {n_visible} visible GPU(s) (RCP_SHARE_GPU=1 to share them)")
    if n == 1:
        return 1, None
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port or free_port()),
           os.path.abspath(__file__)] + list(argv)
    return n, cmd


def devices_used(world, n_visible, share):
    """Distinct GPUs the ranks run on (rank r on device r % n_visible when they share)."""
    if not share:
        return world
    return len({r % max(n_visible, 1) for r in range(world)})


def main():
    args = parse()
    n_visible = torch.cuda.device_count()
    share = os.environ.get("RCP_SHARE_GPU") == "1"
    world, cmd = launch_plan(args, os.environ, n_visible, sys.argv[1:])
    if cmd is not None:
        # N ranks as children; this process has not touched the GPU (no exec after GPU init)
        log("bench.py: starting", " ".join(cmd))
        env = dict(os.environ)
        if share:
            env.setdefault("RCP_DIST_BACKEND", "gloo")
        sys.exit(__import__("subprocess").call(cmd, env=env))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = world > 1
    # rehearsal of the N > 1 path on fewer GPUs: RCP_SHARE_GPU=1 puts several ranks on one device
    # and (RCP_DIST_BACKEND=gloo, its default then: RCCL needs one rank per GPU) the barrier /
    # max-reduction / gather on the host
    backend = os.environ.get("RCP_DIST_BACKEND", "gloo" if share else "nccl")
    if share:
        local = local % max(n_visible, 1)
    if dist:
        import torch.distributed as tdist
        torch.cuda.set_device(local)
        if backend == "nccl":
            tdist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
        else:  # (gloo prints its connection lines on stdout: sent to stderr, the JSON line stays alone)
            sys.stdout.flush()
            fd = os.dup(1)
            os.dup2(2, 1)
            try:
                tdist.init_process_group(backend)
                tdist.barrier()
            finally:
                os.dup2(fd, 1)
                os.close(fd)
    dev = f"cuda:{local}"
    torch.cuda.set_device(local)

    from recoup_amd.engine import Plan, ReadSet

    t0 = time.time()
    data, rows_all, bins, ovl_all = workload(args, dev)
    R_total = rows_all.n_rows
    n_reads_total = int(data["reads"][1].numel())
    s_rank, s_world = rank, world
    if args.sim_shard:
        s_rank, s_world = (int(x) for x in args.sim_shard.split("/"))
    lo, hi, cuts = shard_of(rows_all, ovl_all, s_world, s_rank)
    rows = subset_rows(rows_all, lo, hi) if s_world > 1 else rows_all
    reads = reads_for_rows(data["reads"], rows, len(data["seqlen"])) if s_world > 1 else data["reads"]
    if world > 1 and not args.verify_gather:
        data["reads"] = None  # the full read set is not kept on this rank
    R = rows.n_rows
    n_reads = int(reads[1].numel())
    torch.cuda.synchronize()
    log(f"[rank {rank}] data {args.config}: shard rows [{lo}, {hi}) of {R_total}, {n_reads} of {n_reads_total} "
        f"reads in {time.time() - t0:.1f}s")
    shards = [{"rank": rank, "device": local, "rows": [lo, hi], "reads": n_reads}]
    if dist:  # every rank's shard, for the line rank 0 prints
        got = [None] * world
        tdist.all_gather_object(got, shards[0])
        shards = got

    t1 = time.time()
    rs = ReadSet(*reads, data["seqlen"], device=local)
    tp = time.time()
    plan = Plan(rs, rows, bins, out_ld="padded", kernel=args.kernel)  # whole 128-B lines per 16-row column segment
    plan_s = time.time() - tp
    B = plan.n_cols
    out = plan.empty_output()
    valid = torch.empty(max(R, 1), dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    log(f"[rank {rank}] readset + plan in {time.time() - t1:.1f}s (plan {plan_s * 1e3:.1f} ms), info {plan.info}")

    # ---- samples in flight: D DISTINCT samples (independent read sets over the same region
    # table: profileMatrix's loop over a recoup input list, R/profile.R:13-98), one plan each, on
    # D HIP streams; step k is one complete pass of sample k % D.  Passes are independent, so
    # with D = 2 one sample's locate / heavy launches and its pileup's tail overlap another's
    # pileup.  D = 1 (the default) is one sample, pass after pass.
    # D = 1 runs `plan` (built alone); D > 1 runs one plan per sample built with
    # concurrent = dmax (rcp_plan_opts.concurrent: persistent pileup grids leave 1/8 of the
    # workgroup slots to the other samples' locate / heavy launches)
    plans, outs, valids, rsets = [plan], [out], [valid], [rs]
    streams = [torch.cuda.current_stream()]
    dmax = 4 if args.inflight == "auto" else int(args.inflight)
    if dmax > 1:
        for k in range(1, dmax):
            dk = workload(args, dev, sample=k)[0]
            rk = reads_for_rows(dk["reads"], rows, len(dk["seqlen"])) if s_world > 1 else dk["reads"]
            rsets.append(ReadSet(*rk, dk["seqlen"], device=local))
            del dk, rk
            valids.append(torch.empty(max(R, 1), dtype=torch.uint8, device=dev))
        plans = [Plan(rsets[k], rows, bins, out_ld="padded", concurrent=dmax, kernel=args.kernel) for k in range(dmax)]
        outs = [p.empty_output() for p in plans]
        streams = [torch.cuda.Stream(device=dev) for _ in range(dmax)]

    def passes(D, n):
        for k in range(n):
            if D == 1:
                plan.execute(out, valid, stream=streams[0])
                continue
            i = k % D
            plans[i].execute(outs[i], valids[i], stream=streams[i])

    # ---- warmup + correctness gate
    passes(1, max(args.warmup, 1))
    if dmax > 1:
        passes(len(plans), max(args.warmup, len(plans)))
    for p in plans + [plan]:
        p.status()
    tune = {}
    for d in ([1] + ([2, 3, 4] if args.inflight == "auto" else [])):
        torch.cuda.synchronize()
        t = time.perf_counter()
        passes(d, max(args.steps, 10))
        torch.cuda.synchronize()
        tune[d] = (time.perf_counter() - t) / max(args.steps, 10) * 1e3
    if dist and len(tune) > 1:  # one D for every rank: the per-D times, max over ranks
        tt = torch.tensor([tune[k] for k in sorted(tune)], dtype=torch.float64,
                          device=dev if backend == "nccl" else "cpu")
        tdist.all_reduce(tt, op=tdist.ReduceOp.MAX)
        tune = {k: float(v) for k, v in zip(sorted(tune), tt.tolist())}
    D = min(tune, key=tune.get) if args.inflight == "auto" else len(plans)

    # ---- timed region: exactly K steps between barrier + synchronize
    if dist:
        tdist.barrier()
    torch.cuda.synchronize()
    ts = time.perf_counter()
    passes(D, args.steps)
    torch.cuda.synchronize()
    if dist:
        tdist.barrier()
    elapsed = time.perf_counter() - ts
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        elapsed = float(t.item())
    for p in plans + [plan]:
        p.status()
    # every sample the timed passes computed, checked bit for bit against an independent plan of
    # its readset on the general pileup kernel (sample 0 is also checked against the oracle below)
    inflight_check = []
    for i in range(D):
        ref_plan = Plan(rsets[i], rows, bins, kernel="general", out_ld="padded")
        ref_out = ref_plan.execute()
        ref_plan.status()
        got = (outs[i] if D > 1 else out)[:, :R]
        inflight_check.append(bool(torch.equal(got.view(torch.int64), ref_out[:, :R].view(torch.int64))))
        del ref_plan, ref_out

    # ---- per-kernel durations with HIP events on the launch stream.  A short sleep kernel first
    # keeps the stream busy while the host enqueues the three stages, so a stage's interval is its
    # kernels' time, not the host's launch latency (a folded plan's locate stage is empty: its
    # pileup would otherwise start only when the host gets to it)
    stream = torch.cuda.current_stream()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    kt = np.zeros(3)
    for _ in range(args.steps):
        gpu_sleep(200e-6)
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
    # the pileup kernel alone: 8 launches back to back between two events (each stage interval
    # above also holds ~9 us of event overhead -- the empty stages' own intervals -- which is a
    # third of a C2 launch); every pileup kernel resets its own work counters, so the stage can
    # run again on the same locate outputs
    k_pile = 0.0
    for _ in range(max(1, args.steps // 4)):
        gpu_sleep(400e-6)
        ev[0].record(stream)
        for _ in range(8):
            plan.execute_stages(2, out)
        ev[1].record(stream)
        torch.cuda.synchronize()
        k_pile += ev[0].elapsed_time(ev[1]) / 8
    k_pile /= max(1, args.steps // 4)
    plan.status()
    heavy = plan.heavy_rows()

    # ---- reassembly of the R x B matrix (not in `value`): one all_gather of each rank's
    # column-major block, padded to the largest shard, then placement into region order
    gather = None
    if dist:
        gather, full = gather_matrix(tdist, backend, out, R, B, cuts, dev, R_total)
        if args.verify_gather and rank == 0:
            rs_all = ReadSet(*data["reads"], data["seqlen"], device=local)
            ref = Plan(rs_all, rows_all, bins).execute()
            torch.cuda.synchronize()
            gather["parity_vs_single_gpu"] = bool(torch.equal(full.to(ref.device).view(torch.int64),
                                                              ref.view(torch.int64)))
            del rs_all, ref
        del full

    units = R_total * B  # region-bins per step of the whole job
    if args.sim_shard:
        units = R * B  # a rehearsal of one shard: its own region-bins
    value = units * args.steps / elapsed
    ovl = int(np.asarray(ovl_all)[lo:hi].sum())
    # 8 B per overlapping (read, segment) + 16 B per region + 8 B per further segment
    # of a multi-range row + the f64 output written once (this rank's shard)
    n_seg = len(rows.start)
    bytes_pileup = 8 * ovl + 16 * R + 8 * (n_seg - R) + 8 * R * B
    if args.config == "c3":  # + 4 R (B + 1): the per-row bin tables of non-uniform (R-RNG) layouts
        bytes_pileup += 4 * R * (B + 1)
    achieved = bytes_pileup / (k_pile * 1e-3) / 1e9
    # the same with the bytes the kernel actually streams per read: 4 for reads of one width whose
    # starts alone the kernel loads (C2, C5; C4's binned lean kernel loads the pairs)
    rb = int(plan.info.get("read_bytes", 8))
    bytes_streamed = bytes_pileup - (8 - rb) * ovl
    kernel = PILEUP_KERNELS[plan.info["pileup_kernel"]]
    traffic = load_traffic(args.traffic or os.path.join(ROOT, "profiles", f"traffic_{args.config}.json"), args,
                           kernel, R, n_reads, world)
    step_ms = elapsed / args.steps * 1e3

    # ---- end to end once (not `value`): what a host caller (the R shim's rcp_profile) pays --
    # host read arrays -> H2D + device sort (readset), plan, one pass, D2H of the matrix
    e2e = None
    if not args.no_e2e:
        e2e = end_to_end(reads, data["seqlen"], rows, bins, local, R * B)
        if dist:
            t = torch.tensor([e2e["ms"]], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
            tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
            e2e["ms"] = float(t.item())
            e2e["region_bins_per_s"] = units / (e2e["ms"] * 1e-3)
            e2e["note"] += "; per rank on its shard, max over ranks"

    # ---- CPU baseline (rank 0, N = 1): the oracle on a bounded sample of the same workload
    cpu = None
    parity = None
    if rank == 0 and world == 1 and not args.no_cpu and not args.sim_shard:
        cpu, parity = cpu_baseline(args, data, rows, bins, plan, B)

    if rank == 0:
        res = {
            "metric": "region-bins/sec (profileMatrix)",
            "value": value,
            "unit": "region-bins/s",
            "n_gpus": world,
            "devices_used": devices_used(world, n_visible, share),
            "shared_gpu": share,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": step_ms,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic",
            "config": {
                "workload": WORKLOADS[args.config],
                "regions": R_total, "bins": B, "reads": n_reads_total, "samples": D,
                "parallelism": f"region-sharded x{world}: one contiguous region shard per GPU, balanced by "
                               f"overlapping reads; no data-path collective",
                "rank0_shard": {"regions": R, "reads": n_reads, "sim_shard": args.sim_shard},
                "shards": shards,
                "inflight": D,
                "inflight_note": "samples in flight on separate HIP streams: D distinct samples (independent "
                                 "read sets, same regions), every step one complete pass of one sample (D > 1: "
                                 "plans built with rcp_plan_opts.concurrent, D = 1: a plan built alone); rank 0's "
                                 "ms per pass by D: " + json.dumps({str(k): round(v, 4) for k, v in tune.items()}),
                "single_pass_ms": tune[1],
            },
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBPS, "traffic": traffic,
                         "kernel": kernel,
                         "algorithmic_bytes_per_launch": bytes_pileup,
                         "read_bytes": rb,
                         "frac_streamed_bytes": bytes_streamed / (k_pile * 1e-3) / 1e9 / HBM_PEAK_GBPS,
                         "streamed_bytes_note": "frac with the bytes per read the kernel loads (read_bytes) instead of "
                                                "SURVEY 8(d)'s 8: the start-only stream of reads of one width",
                         "kernel_ms": k_pile,
                         "kernel_ms_note": "the pileup stage's kernel(s) per launch, 8 launches back to back between "
                                           "two HIP events on the launch stream (kernel_ms below: one stage per "
                                           "event pair, each interval with ~9 us of event overhead)",
                         "step_frac": bytes_pileup / (step_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS if world == 1 else None},
            "cpu_baseline": cpu,
            "e2e": e2e,
            "gather": gather,
            "kernel_ms": {"locate": kt[0], "pileup": kt[1], "interp": kt[2]},
            "heavy_rows": heavy,
            "n_overlaps": ovl,
            "plan_ms": plan_s * 1e3,
            "parity_sample": parity,
            "inflight_check": {"samples": D, "equal_to_general_kernel": inflight_check},
        }
        print(json.dumps(res), flush=True)
    if dist:
        tdist.destroy_process_group()


def gather_matrix(tdist, backend, out, R, B, cuts, dev, R_total, reps=3):
    """Reassemble the full R x B column-major matrix on every rank: all_gather of each rank's
    (B, n_r) block padded to the largest shard (RCCL over xGMI on GPU ranks), then one device
    copy per rank block into region order.  Returns timing (max over ranks) and bytes."""
    world = len(cuts) - 1
    nmax = int(np.max(np.diff(cuts)))
    on_gpu = backend == "nccl"
    blk = torch.zeros((B, nmax), dtype=torch.float64, device=dev if on_gpu else "cpu")
    recv = torch.empty((world, B, nmax), dtype=torch.float64, device=blk.device)
    full = torch.empty((B, R_total), dtype=torch.float64, device=blk.device)
    times = []
    for _ in range(reps):
        tdist.barrier()
        torch.cuda.synchronize()
        t = time.perf_counter()
        blk[:, :R].copy_(out[:, :R], non_blocking=True)
        if on_gpu:
            tdist.all_gather_into_tensor(recv, blk)
        else:
            tdist.all_gather(list(recv.unbind(0)), blk)
        for r in range(world):
            full[:, cuts[r]:cuts[r + 1]].copy_(recv[r, :, :cuts[r + 1] - cuts[r]], non_blocking=True)
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t)
    ms = float(np.mean(times[1:] if len(times) > 1 else times)) * 1e3
    tt = torch.tensor([ms], dtype=torch.float64, device=blk.device)
    tdist.all_reduce(tt, op=tdist.ReduceOp.MAX)
    return {"ms": float(tt.item()), "bytes_per_rank_received": (world - 1) * B * nmax * 8,
            "backend": "rccl" if on_gpu else backend,
            "note": "all_gather_into_tensor of padded (B, R/N) blocks + placement; not part of value"}, full


def end_to_end(reads, seqlen, rows, bins, local, units, reps=3, rle=True):
    """Host-to-host passes through the C ABI entry points the R shim binds, timed in two
    phases: rcp_readset_create from host read arrays (H2D + device sort + stream index), then
    rcp_profile (plan + one pass + D2H of the R column-major matrix into caller-owned host
    memory, already touched as R's allocMatrix result is).  Two input forms:
      * "sorted_runs" -- what R holds for a coordinate-sorted BAM (readGAlignments keeps file
        order, R/ranges.R:111-132): reads in (chromosome, start) order, seqnames as the runs of
        its Rle (the shim passes runValue / runLength) and the widths as runs of Rle(width(x))
        when they are few (r/R/rcp.R: at most one run per 4 reads, else the end vector) --
        the headline e2e;
      * "any_order" -- the same reads in generation order, one chromosome code per read.
    `reps` calls each; `ms` is the median call, `first_call_ms` the first (it also pays the
    pinned staging buffers and the first big device allocations).  Reported beside `value`,
    never as it."""
    from recoup_amd.engine import ReadSet, profile_host
    chrom, start, end, strand = reads
    order = torch.argsort((chrom.to(torch.int64) << 32) | start.to(torch.int64))
    sc = chrom[order]
    rv, rl = torch.unique_consecutive(sc, return_counts=True)
    sw = (end[order] - start[order] + 1).to(torch.int32)
    wv, wl = torch.unique_consecutive(sw, return_counts=True)
    ends = ((wv.cpu().numpy(), wl.to(torch.int64).cpu().numpy()) if wv.numel() <= sw.numel() // 4
            else end[order].cpu().numpy())
    # the same reads in generation order, in the form r/R/rcp.R hands them over: one chromosome
    # code per read (seqnames has about one run per read), the widths as runs when they are few
    # (C4: one width), else one end per read
    aw = (end - start + 1).to(torch.int32)
    awv, awl = torch.unique_consecutive(aw, return_counts=True)
    a_ends = ((awv.cpu().numpy(), awl.to(torch.int64).cpu().numpy()) if awv.numel() <= aw.numel() // 4
              else end.cpu().numpy())
    del aw, awv, awl
    forms = {
        "sorted_runs": [(rv.to(torch.int32).cpu().numpy(), rl.to(torch.int64).cpu().numpy()),
                        start[order].cpu().numpy(), ends, strand[order].cpu().numpy()],
        "any_order": [chrom.cpu().numpy(), start.cpu().numpy(), a_ends, strand.cpu().numpy()],
        "any_order_ends": [x.cpu().numpy() for x in reads],
    }
    n_wruns = int(wv.numel()) if isinstance(ends, tuple) else None
    del order, sc, sw, wv, wl
    out = np.zeros((bins.n_cols, rows.n_rows))  # R's matrix: allocated + touched before the call
    valid = np.zeros(max(rows.n_rows, 1), np.uint8)
    res = {}
    for name, host in forms.items():
        calls = []
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            rs = ReadSet(*host, seqlen, device=local)
            t1 = time.perf_counter()
            profile_host(rs, rows, bins, out, valid)
            t2 = time.perf_counter()
            del rs
            calls.append(((t2 - t0) * 1e3, (t1 - t0) * 1e3, (t2 - t1) * 1e3))
        med = sorted(calls)[len(calls) // 2]
        res[name] = {"ms": med[0], "region_bins_per_s": units / (med[0] * 1e-3),
                     "phases_ms": {"readset_create": med[1], "profile_one_shot": med[2]},
                     "first_call_ms": calls[0][0], "calls_ms": [round(c[0], 2) for c in calls]}
    e2e = one_call(forms["sorted_runs"], seqlen, rows, bins, local, units, out, reps)
    e2e["two_calls"] = res["sorted_runs"]
    e2e["any_order"] = res["any_order"]
    e2e["any_order_ends"] = res["any_order_ends"]
    e2e["samples_pipelined"] = samples_pipelined(forms["sorted_runs"], seqlen, rows, bins, local, units, out, reps)
    if rle:
        e2e["rle_path"] = rle_path(forms["sorted_runs"], seqlen, rows, bins, local, units, out, reps)
    e2e["width_runs"] = n_wruns
    e2e["note"] = ("host reads -> host matrix through the C ABI, PCIe both ways. ms: one rcp_profile_reads call "
                   "(profileMatrixFromReads), reads coordinate-sorted with seqnames runs (a sorted BAM) and width "
                   "runs when few (width_runs: their count; null = per-read ends), streamed in row blocks; "
                   "two_calls: rcp_readset_create then rcp_profile (phases_ms); any_order: the two calls on "
                   "unsorted reads as r/R/rcp.R hands them over (one chromosome code per read, width runs when "
                   "few); any_order_ends: the same with one end per read")
    return e2e


def one_call(host, seqlen, rows, bins, local, units, fused, reps):
    """The headline e2e: profileMatrix straight from one sample's host reads in one C ABI call,
    as r/R/rcp.R's profileMatrixFromReads makes it (rcp_profile_reads): coordinate-sorted reads
    stream through the GPU in row blocks -- block b's slice of the reads goes up while block b - 1's
    rows of the matrix come down.  `fused`: the matrix of the two-call sequence (readset_create +
    rcp_profile), which this must equal bit for bit."""
    from recoup_amd.engine import profile_reads
    out = np.zeros((bins.n_cols, rows.n_rows))
    calls = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        res = profile_reads([host], seqlen, rows, bins, local, [out])
        calls.append((time.perf_counter() - t0) * 1e3)
    med = sorted(calls)[len(calls) // 2]
    return {"ms": med, "region_bins_per_s": units / (med * 1e-3), "first_call_ms": calls[0],
            "calls_ms": [round(c, 2) for c in calls],
            "equal_two_calls": bool(np.array_equal(res[0][0].T.view(np.int64), fused.view(np.int64)))}


def samples_pipelined(host, seqlen, rows, bins, local, units, fused, reps, n_samples=3):
    """profileMatrix straight from the reads of an input list of samples (r/R/rcp.R
    profileMatrixFromReads -> rcp_profile_reads): sample k + 1's reads go up while sample k's
    matrix comes down (both PCIe directions; the sequential e2e above uses one at a time).  The
    samples reuse one sample's host arrays (the timing does not depend on their values); `ms` is
    per sample, the median of `reps` calls of n_samples samples each."""
    from recoup_amd.engine import profile_reads
    outs = [np.zeros((bins.n_cols, rows.n_rows)) for _ in range(n_samples)]
    calls = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        res = profile_reads([host] * n_samples, seqlen, rows, bins, local, outs)
        calls.append((time.perf_counter() - t0) * 1e3 / n_samples)
    med = sorted(calls)[len(calls) // 2]
    return {"ms": med, "region_bins_per_s": units / (med * 1e-3), "samples": n_samples,
            "calls_ms_per_sample": [round(c, 2) for c in calls],
            "equal_one_shot": bool(all(np.array_equal(m.T.view(np.int64), fused.view(np.int64)) for m, _ in res)),
            "note": "rcp_profile_reads: readset upload + build of sample k+1 beside the pass and matrix download "
                    "of sample k (both PCIe directions); per-sample time"}


def rle_path(host, seqlen, rows, bins, local, units, fused, reps):
    """The path recoup() takes through the R wrappers (r/R/rcp.R) with saveParams$coverage =
    TRUE, the default (R/util.R:459-461): coverageRef -> calcCoverage -> rcp_coverage_rle (GPU
    pileup + GPU run-length encoding, runs copied to the host: the `$coverage` list of Rle,
    R/coverage.R:171-173), then profileMatrix -> binCoverageMatrix / baseCoverageMatrix ->
    rcp_profile_rle over those host run arrays (R/recoup.R:551-597, R/profile.R:100-212).
    Phases per call: readset_create, coverage_rle (incl. the D2H of the runs), profile_rle
    (H2D of the runs, the profile kernel, D2H of the matrix).  The matrix is checked bit-equal
    to the fused pass's (``fused``, the host matrix end_to_end just filled)."""
    from recoup_amd.engine import ReadSet, coverage_rle_kept, profile_rle_arrays
    out = np.zeros((rows.n_rows, bins.n_cols), order="F")
    up = np.zeros((rows.n_rows, bins.n_cols), order="F")
    calls = []
    n_runs = None
    upload_ms = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        rs = ReadSet(*host, seqlen, device=local)
        t1 = time.perf_counter()
        kept = coverage_rle_kept(rs, rows)
        run_off, values, lengths, valid = kept.copy()  # the list of Rle R builds
        t2 = time.perf_counter()
        kept.profile(bins, out)  # profileMatrix of that unchanged list: its runs on the device
        t3 = time.perf_counter()
        # the same list after it changed (an element replaced, save / load): its runs uploaded
        profile_rle_arrays(run_off, lengths, values, (valid == 0).astype(np.uint8), bins, local, up)
        upload_ms.append((time.perf_counter() - t3) * 1e3)
        del rs
        kept.close()
        n_runs = int(run_off[-1])
        # the host runs (0.8 GB on C4) are released between calls, outside the timed phases: R
        # frees a finished call's vectors at its garbage collection, not inside the next call
        # (unmapping them inside `coverage_rle` of the next call cost ~35 ms)
        del run_off, values, lengths, valid
        calls.append(((t3 - t0) * 1e3, (t1 - t0) * 1e3, (t2 - t1) * 1e3, (t3 - t2) * 1e3))
    med = sorted(calls)[len(calls) // 2]
    return {"ms": med[0], "region_bins_per_s": units / (med[0] * 1e-3),
            "phases_ms": {"readset_create": med[1], "coverage_rle": med[2], "profile_rle": med[3]},
            "calls_ms": [round(c[0], 2) for c in calls], "n_runs": n_runs,
            "run_bytes": 8 * n_runs, "equal_fused": bool(np.array_equal(out.T.view(np.int64), fused.view(np.int64))),
            "profile_rle_upload_ms": sorted(upload_ms)[len(upload_ms) // 2],
            "equal_upload": bool(np.array_equal(up.view(np.int64), out.view(np.int64))),
            "note": "recoup()'s default R path: rcp_coverage_rle (GPU pileup + RLE, runs to the host: the list of "
                    "Rle) then profileMatrix of that unchanged list from its runs still on the device "
                    "(rcp_profile_cov; r/R/rcp.R keeps them beside the list); profile_rle_upload_ms: the same "
                    "profile of the host runs uploaded again (rcp_profile_rle: a list that changed, or was "
                    "loaded); equal_fused: bit-equal to the fused rcp_profile matrix"}


def cpu_baseline(args, data, rows, bins, plan, B):
    """The oracle (C restatement of the reference's per-region dataflow, multithreaded over
    regions like cmclapply with rc = NULL) on the first --cpu-regions rows, repeated for about
    --cpu-seconds; multi-range rows (C3) go through the oracle's per-group coverage + splitVector."""
    from oracle import oracle as o
    from recoup_amd.engine import RowTable
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
    threads, basis = host_cores()
    single = bool(np.all(np.diff(rows.seg_off[:m + 1]) == 1)) and len(bins.parts) == 1
    if single:
        mask = o.Mask.from_ranges(rows.chrom[:m], rows.start[:m], rows.end[:m], rows.strand[:m])
        nb = int(bins.n_bins[0])

        def run():
            if nb > 0:
                return o.profile_part(ix, mask, nb, nthreads=threads)
            return o.profile_part(ix, mask, 0, ncol=B, nthreads=threads)
    else:
        sub = RowTable(rows.seg_off[:m + 1], rows.chrom[:rows.seg_off[m]], rows.start[:rows.seg_off[m]],
                       rows.end[:rows.seg_off[m]], rows.strand[:rows.seg_off[m]],
                       seg_group=None if rows.seg_group is None else rows.seg_group[:rows.seg_off[m]],
                       group_is_list=rows.group_is_list, ignore_strand=rows.ignore_strand)

        def run():
            return o.profile_rows(ix, sub, bins, nthreads=threads)
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
    parity = parity_check(plan, bins, ref, rvalid, m, single)
    # the same restatement on ONE core (beside the all-cores figure), on the first
    # tenth of the sample's rows so it stays within about --cpu-seconds / 2
    m1 = max(1, m // 10)
    if single:
        mask1 = o.Mask.from_ranges(rows.chrom[:m1], rows.start[:m1], rows.end[:m1], rows.strand[:m1])

        def run1():
            if nb > 0:
                return o.profile_part(ix, mask1, nb, nthreads=1)
            return o.profile_part(ix, mask1, 0, ncol=B, nthreads=1)
    else:
        sub1 = RowTable(rows.seg_off[:m1 + 1], rows.chrom[:rows.seg_off[m1]], rows.start[:rows.seg_off[m1]],
                        rows.end[:rows.seg_off[m1]], rows.strand[:rows.seg_off[m1]],
                        seg_group=None if rows.seg_group is None else rows.seg_group[:rows.seg_off[m1]],
                        group_is_list=rows.group_is_list, ignore_strand=rows.ignore_strand)

        def run1():
            return o.profile_rows(ix, sub1, bins, nthreads=1)
    reps1 = 0
    t = time.perf_counter()
    while True:
        run1()
        reps1 += 1
        if time.perf_counter() - t >= args.cpu_seconds / 2:
            break
    dt1 = (time.perf_counter() - t) / reps1
    cpu = {"value": m * B / dt, "unit": "region-bins/s", "cores": threads, "kind": "port",
           "sample": f"first {m} of {R} rows (all their reads), {B} columns; oracle/ C restatement, "
                     f"{threads} threads over regions ({basis}); mean of {reps} passes, {dt:.3f} s/pass",
           "one_core": {"value": m1 * B / dt1, "cores": 1,
                        "sample": f"first {m1} rows, 1 thread; mean of {reps1} passes, {dt1:.3f} s/pass"},
           "cpu_model": cpu_model()}
    return cpu, parity


def parity_check(plan, bins, ref, rvalid, m, single):
    """The GPU pass of sample 0 against the oracle on the sample's first m rows.  Integer work
    is compared bit for bit: per-base columns exactly; uniform bins (L mod n = 0, no R-RNG
    layout) by their integer numerators -- the int64 bin sums the kernel accumulates, against
    the oracle's mean x bin width, which must itself be an integer -- and the means bitwise
    against numerator / width.  Other layouts (R-RNG enlarged bins, spline / median rows) within
    rtol 1e-9 (north_star's bar for means: 1e-6)."""
    out = plan.empty_output()
    valid = torch.empty(max(plan.n_rows, 1), dtype=torch.uint8, device=out.device)
    bs = torch.empty_like(out, dtype=torch.int64)
    plan.execute(out, valid, bs)
    plan.status()
    gpu = out[:, :m].cpu().numpy().T
    num = bs[:, :m].cpu().numpy().T
    gv = valid[:m].cpu().numpy().astype(bool)
    ok_valid = bool(np.array_equal(gv, np.asarray(rvalid).astype(bool)))
    ref = np.asarray(ref)
    res = {"rows": m, "valid_equal": ok_valid}
    nb = int(bins.n_bins[0]) if single else -1
    lengths = plan.row_lengths()[:m]
    if single and nb == 0:
        res["check"] = "per-base depth bit-exact"
        res["ok"] = ok_valid and bool(np.array_equal(gpu.view(np.int64), ref.view(np.int64)))
    elif single and bins.stat == 0 and nb > 0 and np.all(lengths % nb == 0):
        w = (lengths // nb).astype(np.float64)[:, None]
        rnum = ref * w
        exact = np.abs(rnum - np.rint(rnum)) < 1e-6 * np.maximum(1.0, np.abs(rnum))
        res["check"] = "integer bin numerators bit-exact (int64 GPU sums vs oracle mean x width); means = num / width bitwise"
        res["ok"] = ok_valid and bool(np.all(exact) and np.array_equal(num, np.rint(rnum).astype(np.int64)) and
                                      np.array_equal(gpu.view(np.int64), (num / w).view(np.int64)))
    else:
        # NaN where the reference's neighborhood fill averages four NAs (mean(na.rm = TRUE) of nothing)
        res["check"] = "means within rtol 1e-9 (R-RNG layouts / interpolated / median rows)"
        res["ok"] = ok_valid and bool(np.allclose(gpu, ref, rtol=1e-9, atol=1e-12, equal_nan=True))
    return res


if __name__ == "__main__":
    main()
