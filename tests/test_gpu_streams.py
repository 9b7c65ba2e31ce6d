"""Plans executed on the caller's non-blocking streams while the null stream is busy.

A plan's per-execution work array (tile counters, status words) must be ready before the
plan is returned: its executions run on streams that do not wait for the null stream.  In
round 5 that clear was a null-stream memset -- the symptom was an intermittent wrong block of
rows once several plans ran at once (DESIGN_HISTORY.md, round 5; rcp_host.cpp rcp_plan_create).  Here every
plan is created and executed right behind a long null-stream matmul, several kernels side by
side on their own streams, fresh plans every round (so work arrays come back from the caching
allocator holding another plan's counters), and every output is compared bit for bit with the
same plan's output run alone."""

import numpy as np
import pytest

from tests.test_gpu_random import CHROM_LEN, make_reads, single_rows

pytestmark = pytest.mark.gpu


def test_plans_on_nonblocking_streams_behind_a_busy_null_stream(gpu):
    import torch
    from recoup_amd.engine import Bins, Plan, ReadSet
    rng = np.random.default_rng(6060)
    rs = ReadSet(*make_reads(rng, 200_000), CHROM_LEN, device=0)
    rows = single_rows(rng, 900, 2000)
    cases = [("general", Bins([("whole", 1000)])), ("lean", Bins([("whole", 1000)])),
             ("lean", Bins([("whole", 0, 2000)])), ("bins", Bins([("whole", 200)])),
             ("auto", Bins([("whole", 250)]))]
    ref = [Plan(rs, rows, b, kernel=k).run() for k, b in cases]
    streams = [torch.cuda.Stream(device=0) for _ in cases]
    x = torch.randn(4096, 4096, device="cuda:0")
    n_bad = 0
    for rnd in range(6):
        torch.cuda.synchronize()
        busy = x
        for _ in range(6):  # a few ms of work queued on the null stream
            busy = busy @ x
        plans = [Plan(rs, rows, b, kernel=k) for k, b in cases]
        outs = [p.empty_output() for p in plans]
        for _ in range(2):
            for p, o, st in zip(plans, outs, streams):
                p.execute(o, stream=st)
        torch.cuda.synchronize()
        for (k, _), p, o, a in zip(cases, plans, outs, ref):
            p.status()
            got = o.cpu().numpy()[:, :rows.n_rows].view(np.uint64)
            want = np.ascontiguousarray(a[0]).T.view(np.uint64)
            if not np.array_equal(got, want):
                n_bad += 1
                print(f"round {rnd} kernel {k}: {int((got != want).any(axis=0).sum())} rows differ")
        del plans, outs
    assert n_bad == 0
