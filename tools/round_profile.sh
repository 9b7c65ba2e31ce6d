#!/bin/bash
# One round's measurement set (run on the GPU box):  tools/round_profile.sh OUTDIR
#   PMC traffic of the C4 pileup (separate --pmc passes), the C4 bench line with that traffic,
#   the rocprofv3 kernel-trace summary of the same bench command, and the other configs' lines.
set -e
OUT=${1:-gpurun_out/round}
mkdir -p "$OUT"
export TMPDIR=/tmp
PASSES=traffic bash tools/pmc.sh "$OUT/pmc" c4
python3 tools/pmc_traffic.py "$OUT/pmc" "$OUT/traffic_c4.json" "${CALIB:-profiles/fetch_calib.json}"
timeout -k 10 600 python3 bench.py --traffic "$OUT/traffic_c4.json" > "$OUT/c4_bench.json" 2> "$OUT/c4_bench.err"
cat "$OUT/c4_bench.json"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o bench -- \
    python3 bench.py --no-cpu --no-e2e --inflight 1 --traffic "$OUT/traffic_c4.json" > "$OUT/c4_bench_under_rocprof.json" 2> "$OUT/prof.err"
for c in c2 c3 c5; do
    timeout -k 10 600 python3 bench.py --config $c > "$OUT/${c}_bench.json" 2> "$OUT/${c}_bench.err"
    cat "$OUT/${c}_bench.json"
done
