"""Config C3 (coverageRnaRef spliced) at test scale: genes with exon lists and flanks, spliced
mate alignments split into blocks (synthetic.c3), upstream 50 / centre 500 / downstream 50
bins -- variable-length rows, R-RNG bin layouts, interpolated short genes, duplicate hits of
reads spanning exons.  HIP path vs the CPU oracle (tests/oracle_rows.py)."""
import numpy as np
import pytest

import synthetic
from recoup_amd.engine import Bins
from tests.test_gpu_random import run_case

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def c3(gpu):
    # a small genome so that the uniform 30 % of the reads reach every 2 kb flank
    d = synthetic.c3(device="cuda:0", seed=7, n_genes=600, n_pairs=300_000, genome=[9_000_000, 6_000_000])
    reads = tuple(t.cpu().numpy() for t in d["reads"])
    return d, reads


@pytest.mark.parametrize("stat", ["mean", "median"])
@pytest.mark.parametrize("ignore_strand", [True, False])
def test_c3_profile(c3, stat, ignore_strand):
    d, reads = c3
    rows = synthetic.rna_rows(d, ignore_strand=ignore_strand)
    bins = Bins([("upstream", 50), ("center", 500), ("downstream", 50)], flank=d["flank"], stat=stat)
    (mat, valid), (exp, ev, cov) = run_case(reads, d["seqlen"], rows, bins)
    np.testing.assert_array_equal(valid, ev.astype(bool))
    assert valid.sum() > 0.5 * len(valid)
    lens = np.array([len(c) for c in cov if c is not None])
    assert (lens - 4000 < 500).any() and (lens - 4000 > 500).any()  # interpolated and RNG-layout centres
    np.testing.assert_allclose(mat, exp, rtol=1e-9, atol=1e-12)


def test_c3_overlap_count(c3):
    """The harness's independent overlap count (bench roofline bytes) matches the oracle's
    per-segment candidate count on the row table."""
    d, reads = c3
    rows = synthetic.rna_rows(d)
    import torch
    dev_reads = tuple(torch.as_tensor(x, device="cuda:0") for x in reads)
    cnt = synthetic.n_overlaps_segments(dev_reads, rows.chrom, rows.start, rows.end)
    s, e = reads[1], reads[2]
    for j in range(0, len(rows.start), 97):
        m = (reads[0] == rows.chrom[j]) & (s <= rows.end[j]) & (e >= rows.start[j])
        assert cnt[j] == m.sum()
