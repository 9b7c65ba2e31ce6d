"""Summarise a rocprofv3 kernel_stats.csv: the RLE-path and pileup kernels (avg us per call)."""
import csv
import sys

KEYS = ("rle_tile", "rle_interp", "rle_emit", "rle_count", "cov_runs", "pileup_kernel<false, true", "pileup_lean", "locate",
        "scan_impl<(rocprim::ROCPRIM_400200_NS::detail::lookback_scan_determinism)0, true, true, rocprim::ROCPRIM_400200_NS::default_config, hipcub")
for path in sys.argv[1:]:
    print(path)
    for r in csv.DictReader(open(path)):
        if any(k in r["Name"] for k in KEYS):
            print(f"  {r['Name'][:70]:70s} calls {r['Calls']:>4s} avg {float(r['AverageNs']) / 1e3:9.1f} us")
