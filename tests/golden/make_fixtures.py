"""Regenerate the committed golden fixtures (run in the build container only).

Step 1 (inputs): decode the reference's own test fixture
``/root/reference/data/recoup_test_data.rda`` (documented in
``man/recoup_test_data.Rd:1-39``) with the data-only XDR reader ``rdata.py`` and write
``recoup_test_data.npz`` — plain arrays, no code.

Step 2 (expected outputs): run the CPU oracle (``oracle/``, a restatement of
``R/coverage.R`` + ``R/profile.R`` + ``R/util.R:15-85``) on the C1 configuration of
``inst/unitTests/test_recoup.R:4-26`` and write ``c1_expected.npz``.  These expected
vectors come from the restatement, not from executed R (R is absent here, see
DESIGN.md §2), so they pin the HIP path to the oracle; the oracle itself is
pinned by R's published RNG known answers and the SURVEY Appendix B sanity numbers.

Usage:  python tests/golden/make_fixtures.py [--inputs] [--expected]
"""
import argparse
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
RDA = "/root/reference/data/recoup_test_data.rda"

STRAND_CODE = {"+": 0, "-": 1, "*": 2}


def make_inputs():
    sys.path.insert(0, HERE)
    import rdata

    d = rdata.read_rda(RDA)
    out = {}
    for i, s in enumerate(d["test.input"].value):
        fields = {n: v for n, v in zip(s.a("names").value, s.value)}
        g = rdata.granges_to_dict(fields["ranges"])
        assert list(np.unique(g["seqnames"])) == ["chr12"]
        out[f"s{i}_id"] = np.array(fields["id"].value[0])
        out[f"s{i}_name"] = np.array(fields["name"].value[0])
        out[f"s{i}_start"] = g["start"].astype(np.int32)
        out[f"s{i}_end"] = g["end"].astype(np.int32)
        out[f"s{i}_strand"] = np.array([STRAND_CODE[x] for x in g["strand"]], dtype=np.int8)
        out[f"s{i}_seqlevels"] = g["seqlevels"]
        out[f"s{i}_seqlengths"] = g["seqlengths"]
    gen = rdata.dataframe_to_dict(d["test.genome"])
    for k in ("chromosome", "start", "end", "gene_name", "strand"):
        out[f"genome_{k}"] = gen[k]
    des = rdata.dataframe_to_dict(d["test.design"])
    out["design_rownames"] = des["_rownames"]
    out["design_strand"] = des["strand"]
    out["design_RNA_status"] = des["RNA_status"]
    ex = d["test.exons"]
    ul = rdata.granges_to_dict(ex.a("unlistData"))
    part = ex.a("partitioning")
    out["exons_seqnames"] = ul["seqnames"]
    out["exons_start"] = ul["start"].astype(np.int32)
    out["exons_end"] = ul["end"].astype(np.int32)
    out["exons_strand"] = np.array([STRAND_CODE[x] for x in ul["strand"]], dtype=np.int8)
    out["exons_names"] = ul["names"]
    out["exons_part_end"] = part.a("end").value.astype(np.int32)
    out["exons_part_names"] = np.array([str(x) for x in part.a("NAMES").value])
    path = os.path.join(HERE, "recoup_test_data.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path), "bytes")


def make_expected():
    sys.path.insert(0, REPO)
    from tests.golden import c1_cases

    res = c1_cases.compute_all_with_oracle()
    path = os.path.join(HERE, "c1_expected.npz")
    np.savez_compressed(path, **res)
    print("wrote", path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--inputs", action="store_true")
    ap.add_argument("--expected", action="store_true")
    a = ap.parse_args()
    if not (a.inputs or a.expected):
        a.inputs = a.expected = True
    if a.inputs:
        make_inputs()
    if a.expected:
        make_expected()
