"""Diagnostics: C4 pileup time per library variant (lean kernel work).

    python tools/diag_lean.py            (RCP_LIB_PATH from env: a variant build from tools/variants.sh)
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.diag_pileup import run  # noqa: E402

if __name__ == "__main__":
    tag = " ".join(f"{k}={os.environ[k]}" for k in ("RCP_LIB_PATH",) if k in os.environ)
    run(f"c4 default [{tag}]")
    if len(sys.argv) > 1 and sys.argv[1] == "both":
        run(f"c4 uniform [{tag}]", enriched=0.0)
