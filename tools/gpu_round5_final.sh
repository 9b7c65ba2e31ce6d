#!/bin/bash
# Round-5 measurement set, in two parts (each well inside one gpurun call):
#   part A: the full GPU suite, smoke, PMC traffic of the C4 and C2 pileup kernels (separate --pmc
#           passes), the C4 bench line with that traffic (e2e included)
#   part B: the rocprofv3 kernel summary of the C4 bench command, the C2 / C3 / C5 lines, the C4 and
#           C5 1/8 shards at D = 1, the streamed host paths (tools/diag_stream.py)
# usage: tools/gpu_round5_final.sh A|B OUTDIR
set -o pipefail
PART=${1:-A}
OUT=${2:-gpurun_out/r05f}
mkdir -p "$OUT"
export TMPDIR=/tmp
CAL=profiles/fetch_calib.json
if [ "$PART" = A ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
  tail -2 "$OUT/tests.log"
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1 && tail -1 "$OUT/smoke.log" || exit 1
  PASSES=traffic timeout -k 10 400 bash tools/pmc.sh "$OUT/pmc_c4" c4 && python3 tools/pmc_traffic.py "$OUT/pmc_c4" "$OUT/traffic_c4.json" $CAL || exit 1
  PASSES=traffic timeout -k 10 400 bash tools/pmc.sh "$OUT/pmc_c2" c2 && python3 tools/pmc_traffic.py "$OUT/pmc_c2" "$OUT/traffic_c2.json" $CAL || exit 1
  timeout -k 10 600 python3 bench.py --traffic "$OUT/traffic_c4.json" > "$OUT/c4_bench.json" 2> "$OUT/c4_bench.err" || exit 1
  python3 -c "
import json; d=json.load(open('$OUT/c4_bench.json')); e=d['e2e']
print('C4', d['value'], d['ms_per_step'], d['config']['single_pass_ms'], d['roofline'])
print('e2e', round(e['ms'],2), e['equal_two_calls'], 'two calls', round(e['two_calls']['ms'],2), 'pipelined', round(e['samples_pipelined']['ms'],2), 'rle', round(e['rle_path']['ms'],2), e['rle_path']['phases_ms'])"
  exit 0
fi
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o bench -- \
    python3 bench.py --no-cpu --no-e2e --inflight 1 > "$OUT/c4_bench_under_rocprof.json" 2> "$OUT/prof.err" || exit 1
for c in c2 c3 c5; do
  extra=""
  [ $c = c2 ] && extra="--traffic $OUT/traffic_c2.json"
  timeout -k 10 400 python3 bench.py --config $c --no-e2e $extra > "$OUT/${c}_bench.json" 2> "$OUT/${c}_bench.err" || exit 1
  python3 -c "import json; d=json.load(open('$OUT/${c}_bench.json')); print('$c', d['value'], d['ms_per_step'], d['config'].get('single_pass_ms'), d['roofline'].get('frac'), d.get('kernel_ms'))"
done
for c in c4 c5; do
  timeout -k 10 300 python3 bench.py --config $c --sim-shard 0/8 --inflight 1 --no-e2e --no-cpu > "$OUT/${c}_shard.json" 2> "$OUT/${c}_shard.err" || exit 1
  python3 -c "import json; d=json.load(open('$OUT/${c}_shard.json')); print('$c shard', d['ms_per_step'], d['config'].get('single_pass_ms'), d.get('kernel_ms'))"
done
timeout -k 10 300 python3 -u tools/diag_stream.py 9 > "$OUT/diag_stream.log" 2>&1 && grep -h "median\|mismatches" "$OUT/diag_stream.log"
