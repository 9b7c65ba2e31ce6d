"""The lean pileup kernel (pile waves + store waves, rcp_kernels.hip rcp_pileup_lean_kernel).

Plans whose rows are all one plain range with uniform power-of-two bins take the lean kernel
(plan info "pileup_kernel" == 1); other mean plans whose chunks fit one wave pass take its
general-bins mode (2: any bin width, R-RNG layouts, exon lists) when opted in (kernel="lean_any").  Each case checks it against the CPU oracle (validity and
means as in test_gpu_random: integer numerators exact, means within 1e-12 relative) and
bit-for-bit against the general kernel on the same plan (kernel="general")."""

import numpy as np
import pytest

from tests.test_gpu_random import CHROM_LEN, check, make_reads, single_rows

pytestmark = pytest.mark.gpu


def plans(reads, seqlen, rows, bins, strand_filter=None, lean_mode=None, heavy_threshold=-1):
    """(lean result, general result, lean kernel id, expected) for one configuration; the lean
    kernel is forced ("lean": these row tables are below AUTO's row floor for binned plans);
    lean_mode "lean_any" opts in to the general-bins mode."""
    from recoup_amd.engine import Plan, ReadSet
    from tests import oracle_rows
    rs = ReadSet(*reads, seqlen, device=0, strand_filter=strand_filter)
    lean = Plan(rs, rows, bins, kernel=lean_mode or "lean", heavy_threshold=heavy_threshold)
    general = Plan(rs, rows, bins, kernel="general", heavy_threshold=heavy_threshold)
    assert general.info["pileup_kernel"] == 0
    r_lean, r_gen = lean.run(), general.run()
    ix = oracle_rows.index_for(reads, seqlen, strand_filter)
    exp = oracle_rows.profile(oracle_rows.row_coverage(ix, rows), bins)
    return r_lean, r_gen, lean.info["pileup_kernel"], exp


def same(a, b):
    np.testing.assert_array_equal(a[1], b[1])
    assert np.array_equal(a[0].view(np.uint64), b[0].view(np.uint64))  # bit-identical doubles


@pytest.mark.parametrize("width,n_bins", [(2000, 1000), (2000, 500), (2000, 125), (4000, 250), (1024, 1024)])
def test_lean_binned(gpu, width, n_bins):
    from recoup_amd.engine import Bins
    rng = np.random.default_rng(300 + n_bins)
    reads = make_reads(rng, 80_000, star_frac=0.1)
    rows = single_rows(rng, 700, width, edge=True)  # NULL rows: negative index, past the end
    rows.start[1], rows.end[1] = 1, width  # (a start at 0 shortens its row: an R-RNG layout)
    lean, gen, kind, exp = plans(reads, CHROM_LEN, rows, Bins([("whole", n_bins)]))
    assert kind == 1
    check(lean, exp)
    same(lean, gen)


def test_lean_per_base_and_flanks(gpu):
    """Per-base parts (C5) and upstream / center / downstream parts of one row table."""
    from recoup_amd.engine import Bins
    rng = np.random.default_rng(41)
    reads = make_reads(rng, 90_000, widths=(30, 90))
    rows = single_rows(rng, 333, 4000)
    for bins in (Bins([("whole", 0, 4000)]),
                 Bins([("upstream", 0, 1000), ("center", 500), ("downstream", 0, 1000)], flank=(1000, 1000))):
        lean, gen, kind, exp = plans(reads, CHROM_LEN, rows, bins)
        assert kind == 1
        check(lean, exp)
        same(lean, gen)


@pytest.mark.parametrize("strand_filter", [None, "+"])
def test_lean_stranded_rows(gpu, strand_filter):
    """ignore.strand = FALSE: up to three candidate streams per row."""
    from recoup_amd.engine import Bins, RowTable
    rng = np.random.default_rng(53)
    reads = make_reads(rng, 70_000, star_frac=0.25)
    r0 = single_rows(rng, 260, 2048)
    rows = RowTable(r0.seg_off, r0.chrom, r0.start, r0.end, r0.strand, ignore_strand=False)
    lean, gen, kind, exp = plans(reads, CHROM_LEN, rows, Bins([("whole", 256)]), strand_filter)
    assert kind == 1
    check(lean, exp)
    same(lean, gen)


@pytest.mark.parametrize("stranded", [False, True])
def test_lean_dense_rows(gpu, stranded):
    """Rows with more reads than positions (C5-like DNase depth, PCR-duplicate stacks): the
    run-merged LDS adds, on both row orientations, per-base and binned, in both layouts."""
    from recoup_amd.engine import Bins, RowTable
    rng = np.random.default_rng(59)
    n = 240_000
    chrom = rng.integers(0, 3, n).astype(np.int32)
    base = np.array([20_000, 30_000, 40_000])[chrom]
    start = base + rng.integers(0, 12_000, n)
    dup = rng.random(n) < 0.3  # duplicate stacks: runs of equal starts and ends
    start[dup] = base[dup] + 4000 + 37 * rng.integers(0, 40, dup.sum())
    width = np.where(dup, 50, rng.integers(20, 80, n))
    reads = (chrom, start.astype(np.int32), (start + width - 1).astype(np.int32),
             rng.integers(0, 3, n).astype(np.int8))
    R = 240
    rc = rng.integers(0, 3, R).astype(np.int32)
    rs_ = np.array([20_000, 30_000, 40_000])[rc] + rng.integers(-500, 10_000, R)
    strand = rng.integers(0, 3, R).astype(np.int8)
    rows = RowTable(np.arange(R + 1), rc, rs_, rs_ + 2047, strand, ignore_strand=not stranded)
    for bins in (Bins([("whole", 0, 2048)]), Bins([("whole", 512)])):
        lean, gen, kind, exp = plans(reads, CHROM_LEN, rows, bins)
        assert kind == 1
        check(lean, exp)
        same(lean, gen)


def test_lean_heavy_rows(gpu):
    """Skewed rows handed over by the heavy slice kernel."""
    from recoup_amd.engine import Bins
    rng = np.random.default_rng(67)
    reads = make_reads(rng, 200_000, widths=(100, 200))
    rows = single_rows(rng, 150, 2000)
    lean, gen, kind, exp = plans(reads, CHROM_LEN, rows, Bins([("whole", 1000)]))
    assert kind == 1
    check(lean, exp)
    same(lean, gen)


def test_lean_kernel_choice(gpu):
    """Power-of-two uniform bins of single-range rows take the lean kernel (1); R-RNG layouts,
    other widths stay on the general kernel (0), exon lists take the row-wave kernel (3), unless the general-bins mode is
    opted in (kernel="lean_any"); medians always stay on the general kernel."""
    from recoup_amd.engine import Bins, Plan, ReadSet, RowTable
    rng = np.random.default_rng(71)
    reads = make_reads(rng, 20_000)
    rs = ReadSet(*reads, CHROM_LEN, device=0)
    rows = single_rows(rng, 50, 2000)
    seg_off = np.array([0, 2, 3], np.int64)
    exons = RowTable(seg_off, np.zeros(3, np.int32), np.array([1000, 3000, 9000]), np.array([1999, 3999, 10999]),
                     np.zeros(3, np.int8), seg_group=np.zeros(3, np.int8), group_is_list=np.array([1, 0, 0, 0], np.uint8))
    for mode, other in (("lean", 0), ("lean_any", 2)):
        assert Plan(rs, rows, Bins([("whole", 150)]), kernel=mode).info["pileup_kernel"] == other   # dif != 0
        assert Plan(rs, rows, Bins([("whole", 200)]), kernel=mode).info["pileup_kernel"] == other   # bs = 10
        # exon lists: the row-wave kernel under auto (tests/test_gpu_rows.py)
        assert Plan(rs, exons, Bins([("whole", 100)]), kernel=mode).info["pileup_kernel"] == (0 if mode == "lean" else 2)
        assert Plan(rs, rows, Bins([("whole", 1000)], stat="median"), kernel=mode).info["pileup_kernel"] == 0
        assert Plan(rs, rows, Bins([("whole", 1000)]), kernel=mode).info["pileup_kernel"] == 1
        assert Plan(rs, rows, Bins([("whole", 1000)]), kernel="general").info["pileup_kernel"] == 0
    # AUTO: exon lists take the row-wave kernel; binned single-range plans below 36000 rows the
    # general kernel, per-base ones the lean kernel at any row count
    assert Plan(rs, exons, Bins([("whole", 100)])).info["pileup_kernel"] == 3
    assert Plan(rs, rows, Bins([("whole", 1000)])).info["pileup_kernel"] == 0
    assert Plan(rs, rows, Bins([("whole", 0, 2000)])).info["pileup_kernel"] == 1


@pytest.mark.parametrize("width,n_bins", [(2000, 150), (4000, 200), (1500, 256), (3000, 64), (2000, 1000)])
def test_lean_general_bins(gpu, width, n_bins):
    """General-bins mode on single-range rows: R-RNG layouts (2000/150), 20-bp bins (C2),
    24-bp-ish layouts, 47-bp bins with layouts; bit-equal to the general kernel."""
    from recoup_amd.engine import Bins
    rng = np.random.default_rng(500 + n_bins)
    reads = make_reads(rng, 80_000, star_frac=0.1)
    rows = single_rows(rng, 400, width, edge=True)
    rows.start[1], rows.end[1] = 1, width  # (a start at 0 would shorten the row)
    lean, gen, kind, exp = plans(reads, CHROM_LEN, rows, Bins([("whole", n_bins)]), lean_mode="lean_any")
    assert kind == (1 if (n_bins, width) == (1000, 2000) else 2)
    check(lean, exp)
    same(lean, gen)


@pytest.mark.parametrize("stranded", [False, True])
def test_lean_general_exon_lists(gpu, stranded):
    """coverageRnaRef rows (flank | exon list | flank) in the general-bins mode: flank bins,
    R-RNG centre layouts, exon-list weights; interpolated short genes stay on the interp kernel."""
    from recoup_amd.engine import Bins, RowTable
    rng = np.random.default_rng(77)
    reads = make_reads(rng, 120_000, widths=(50, 400))
    seg_off, ch, st, en, sd, gr = [0], [], [], [], [], []
    for g in range(150):
        c = int(rng.integers(0, 3))
        pos = int(rng.integers(5000, CHROM_LEN[c] - 60000))
        strand = int(rng.integers(0, 2))
        ex_s, ex_e, p = [], [], pos
        for _ in range(int(rng.integers(1, 9))):
            w = int(rng.integers(30, 500))
            ex_s.append(p)
            ex_e.append(p + w - 1)
            p += w + int(rng.integers(-100, 2000))  # some overlapping exons
        gs, ge = min(ex_s), max(ex_e)
        ls, le = (gs - 1000, gs - 1) if strand == 0 else (ge + 1, ge + 1000)
        rs_, re_ = (ge + 1, ge + 1000) if strand == 0 else (gs - 1000, gs - 1)
        for s_, e_, grp in [(ls, le, 0)] + [(a, b, 1) for a, b in zip(ex_s, ex_e)] + [(rs_, re_, 2)]:
            ch.append(c); st.append(s_); en.append(e_); sd.append(strand); gr.append(grp)
        seg_off.append(len(st))
    rows = RowTable(np.array(seg_off), np.array(ch), np.array(st), np.array(en), np.array(sd),
                    seg_group=np.array(gr), group_is_list=np.array([0, 1, 0, 0]), ignore_strand=not stranded)
    bins = Bins([("upstream", 40), ("center", 100), ("downstream", 40)], flank=(1000, 1000))
    lean, gen, kind, exp = plans(reads, CHROM_LEN, rows, bins, lean_mode="lean_any")
    assert kind == 2
    check(lean, exp, rtol=1e-9, atol=1e-12)
    same(lean, gen)


@pytest.mark.parametrize("chunks", [4, 8])
def test_lean_more_column_chunks(gpu, chunks):
    """rcp_plan_opts.min_col_chunks: the lean plan cut into more column chunks (each streaming
    only its reads through crange) gives the same bits."""
    from recoup_amd.engine import Bins, Plan, ReadSet
    rng = np.random.default_rng(900 + chunks)
    reads = make_reads(rng, 100_000)
    rows = single_rows(rng, 300, 2000)
    rs = ReadSet(*reads, CHROM_LEN, device=0)
    base = Plan(rs, rows, Bins([("whole", 1000)]), kernel="lean")
    more = Plan(rs, rows, Bins([("whole", 1000)]), kernel="lean", min_col_chunks=chunks)
    assert base.info["pileup_kernel"] == 1 and more.info["pileup_kernel"] == 1
    same(more.run(), base.run())


def test_lean_concurrent_plans(gpu):
    """rcp_plan_opts.concurrent: plans built for several samples in flight take 7/8 of the
    persistent grid's workgroup slots; two such plans on two streams give the bits of plans built
    alone (binned and per-base), and a negative value is refused."""
    import torch
    from recoup_amd._lib import RcpError
    from recoup_amd.engine import Bins, Plan, ReadSet
    rng = np.random.default_rng(1234)
    rs = [ReadSet(*make_reads(rng, 120_000), CHROM_LEN, device=0) for _ in range(2)]
    rows = single_rows(rng, 700, 2000)
    for bins in (Bins([("whole", 1000)]), Bins([("whole", 0, 2000)])):
        alone = [Plan(r, rows, bins, kernel="lean").run() for r in rs]
        conc = [Plan(r, rows, bins, kernel="lean", concurrent=2) for r in rs]
        assert all(p.info["pileup_kernel"] == 1 for p in conc)
        outs = [p.empty_output() for p in conc]
        streams = [torch.cuda.Stream(device=0) for _ in conc]
        for _ in range(3):
            for p, o, st in zip(conc, outs, streams):
                p.execute(o, stream=st)
        torch.cuda.synchronize()
        for p, o, a in zip(conc, outs, alone):
            p.status()
            np.testing.assert_array_equal(o.cpu().numpy()[:, :rows.n_rows].view(np.uint64),
                                          np.ascontiguousarray(a[0]).T.view(np.uint64))
    with pytest.raises(RcpError):
        Plan(rs[0], rows, Bins([("whole", 1000)]), concurrent=-1)


@pytest.mark.parametrize("stranded,strand_filter", [(False, None), (True, None), (True, "+")])
@pytest.mark.parametrize("width", [1, 180])
def test_lean_uniform_width_reads(gpu, stranded, strand_filter, width):
    """Reads of one width (fragments extended to fragLen, fixed read lengths): the layout keeps
    their starts alone and the lean kernel streams those (end = start + width - 1 formed when
    added); binned, per-base and heavy rows, both row orientations, edge rows -- bit-equal to
    the general kernel (which reads the (start, end) pairs) and to the oracle.  One read of
    another width turns the start-only stream off (same bits)."""
    from recoup_amd.engine import Bins, RowTable
    rng = np.random.default_rng(1100 + width + stranded)
    reads = make_reads(rng, 150_000, widths=(width, width), star_frac=0.2)
    r0 = single_rows(rng, 300, 2000, edge=True)  # NULL rows: negative index, past the end
    r0.start[1], r0.end[1] = 1, 2000  # (a start at 0 shortens its row: an R-RNG layout)
    rows = RowTable(r0.seg_off, r0.chrom, r0.start, r0.end, r0.strand, ignore_strand=not stranded)
    for bins in (Bins([("whole", 1000)]), Bins([("whole", 0, 2000)]), Bins([("whole", 250)])):
        lean, gen, kind, exp = plans(reads, CHROM_LEN, rows, bins, strand_filter, heavy_threshold=64)
        assert kind == 1
        check(lean, exp)
        same(lean, gen)
    mixed = (reads[0], reads[1], reads[2].copy(), reads[3])
    mixed[2][7] += 1
    lean, gen, kind, exp = plans(mixed, CHROM_LEN, rows, Bins([("whole", 1000)]), strand_filter)
    check(lean, exp)
    same(lean, gen)


@pytest.mark.parametrize("kernel", ["lean", "general"])
def test_dense_bucket_bounds(gpu, kernel):
    """Row edges inside stacks of duplicate reads: the locate searches' buckets hold hundreds of
    reads, so their answers lie past the directory's inline keys (rcp_device.h dir_k) and the
    bisection continues in the read arrays."""
    from recoup_amd.engine import Bins, Plan, ReadSet, RowTable
    from tests import oracle_rows
    rng = np.random.default_rng(77)
    chrom, start, end, strand = make_reads(rng, 20_000)
    piles = np.sort(rng.choice(np.arange(5_000, 80_000, 700), 40, replace=False))
    pc = np.repeat(np.int32(2), 40 * 150)
    ps = np.repeat(piles, 150).astype(np.int32) + rng.integers(0, 3, 40 * 150).astype(np.int32)
    pe = ps + rng.integers(10, 90, ps.size).astype(np.int32)
    pst = rng.integers(0, 2, ps.size).astype(np.int8)
    reads = (np.concatenate([chrom, pc]), np.concatenate([start, ps]), np.concatenate([end, pe]),
             np.concatenate([strand, pst]))
    # rows starting / ending a few bases around each pile (both edges searched inside it)
    off = rng.integers(-60, 60, 4 * 40)
    s = np.repeat(piles, 4) + off
    rows = RowTable.from_ranges(np.full(s.size, 2, np.int32), s, s + 1023, rng.integers(0, 3, s.size).astype(np.int8))
    rs = ReadSet(*reads, CHROM_LEN, device=0)
    ix = oracle_rows.index_for(reads, CHROM_LEN, None)
    cov = oracle_rows.row_coverage(ix, rows)
    for bins in (Bins([("whole", 1024)]), Bins([("whole", 256)])):
        res = Plan(rs, rows, bins, kernel=kernel, heavy_threshold=0).run()
        check(res, oracle_rows.profile(cov, bins))


@pytest.mark.parametrize("mode", ["lean", "lean_any"])
def test_lean_with_interpolated_single_rows(gpu, mode):
    """Single-range rows shorter than their bins among power-of-two-binned ones: the plan stays
    on the lean kernel and the short rows go through the interpolation kernel, which piles them
    from the locate kernel's per-segment ranges -- locate must write them for such plans (a
    regression: fast rows of lean plans once skipped them and profiled as zeros)."""
    from recoup_amd.engine import Bins
    rng = np.random.default_rng(4242)
    reads = make_reads(rng, 100_000)
    rows = single_rows(rng, 300, 2000)
    short = rng.choice(np.arange(2, 300), 40, replace=False)
    rows.end[short[:20]] = rows.start[short[:20]] + 499   # spline: (1000 - 500) / 1000 >= 0.2
    rows.end[short[20:]] = rows.start[short[20:]] + 899   # neighborhood: 0.1 < 0.2
    for bins in (Bins([("whole", 1000)]), Bins([("whole", 1000)], interp="spline")):
        lean, gen, kind, exp = plans(reads, CHROM_LEN, rows, bins, lean_mode=mode)
        assert kind == 1
        assert lean[1][short].all()
        assert (lean[0][short].sum(axis=1) > 0).all()
        check(lean, exp, rtol=1e-9, atol=1e-12)
        same(lean, gen)


@pytest.mark.parametrize("seqlen", ["known", "NA"])
def test_lean_per_base_fold(gpu, seqlen):
    """Per-base lean plans of a small table (one GPU's shard of C5) search their rows' read
    ranges in the kernel: the store wave that claims an item bisects each row's and the chunk's
    bounds, two lanes a row (no locate launch, no heaviest-first item order).  Dense and sparse
    rows, both strands, NULL rows, NA seqlengths, repeated executions: bit-equal to the locate
    path (an explicit heavy threshold keeps it) and the oracle."""
    from recoup_amd.engine import Bins, Plan, ReadSet
    from tests import oracle_rows
    rng = np.random.default_rng(808 + (seqlen == "NA"))
    sl = CHROM_LEN if seqlen == "known" else np.full(3, -1, np.int64)
    reads = make_reads(rng, 200_000, widths=(50, 50))
    rows = single_rows(rng, 400, 4000, edge=True)
    rows.start[1], rows.end[1] = 1, 4000  # (a start at 0 shortens its row: not a per-base row of 4000)
    bins = Bins([("whole", 0, 4000)])
    rs = ReadSet(*reads, sl, device=0)
    fold = Plan(rs, rows, bins, kernel="lean")
    located = Plan(rs, rows, bins, kernel="lean", heavy_threshold=4096)
    assert fold.info["pileup_kernel"] == 1 and fold.info["fold"] == 1, fold.info
    assert located.info["fold"] == 0
    exp = oracle_rows.profile(oracle_rows.row_coverage(oracle_rows.index_for(reads, sl), rows), bins)
    ref = located.run()
    for _ in range(3):
        got = fold.run()
        check(got, exp)
        same(got, ref)
    np.testing.assert_array_equal(fold.validity(), exp[1])
