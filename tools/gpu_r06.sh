#!/bin/bash
# Round-6 GPU steps; each step under its own time limit, chained so that a failure ends the call.
# usage: tools/gpu_r06.sh STEP[,STEP...] OUTDIR
#   tests    the full -m gpu suite
#   smoke    __graft_entry__.smoke()
#   write    tools/write_bench (the column-major output-write floor of C4's matrix)
#   share2   2 ranks sharing the one GPU: bench.py --gpus 2 --verify-gather (C4)
#   c4       the default bench line (C4, cpu baseline and e2e)
#   shards   C4 and C5 1/8 shards at D = 1 (--sim-shard 0/8)
#   prof     rocprofv3 kernel summary of the C4 bench command
#   configs  the C2, C3 and C5 bench lines (no host paths) and their rocprofv3 kernel summaries
set -o pipefail
STEPS=${1:-tests}
OUT=${2:-gpurun_out/r06}
mkdir -p "$OUT"
export TMPDIR=/tmp
has() { [[ ",$STEPS," == *",$1,"* ]]; }
if has tests; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1 || { tail -60 "$OUT/tests.log"; exit 1; }
  tail -2 "$OUT/tests.log"
fi
if has smoke; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1 && tail -1 "$OUT/smoke.log" || exit 1
fi
if has write; then
  timeout -k 10 120 ./tools/write_bench > "$OUT/write_bench.log" 2>&1 || { cat "$OUT/write_bench.log"; exit 1; }
  cat "$OUT/write_bench.log"
fi
if has share2; then
  RCP_SHARE_GPU=1 timeout -k 10 600 python3 bench.py --gpus 2 --verify-gather --no-cpu --no-e2e > "$OUT/share2_c4.json" 2> "$OUT/share2_c4.err" || { tail -30 "$OUT/share2_c4.err"; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('$OUT/share2_c4.json') if l.startswith('{')][-1]); print('share2', d['n_gpus'], d['devices_used'], d['value'], d['ms_per_step'], d['config']['shards'], d['gather'])"
fi
if has c4; then
  timeout -k 10 600 python3 bench.py > "$OUT/c4_bench.json" 2> "$OUT/c4_bench.err" || { tail -30 "$OUT/c4_bench.err"; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/c4_bench.json')); e=d['e2e']
print('C4', d['value'], d['ms_per_step'], d['config']['single_pass_ms'], d['roofline']['frac'], d['roofline']['kernel_ms'])
print('e2e', round(e['ms'],2), e['equal_two_calls'], 'two calls', round(e['two_calls']['ms'],2), 'any_order', round(e['any_order']['ms'],2), e['any_order']['phases_ms'], 'pipelined', round(e['samples_pipelined']['ms'],2), 'rle', round(e['rle_path']['ms'],2), e['rle_path']['phases_ms'], e['rle_path']['equal_fused'])"
fi
if has shards; then
  for c in c4 c5; do
    timeout -k 10 300 python3 bench.py --config $c --sim-shard 0/8 --inflight 1 --no-e2e --no-cpu > "$OUT/${c}_shard.json" 2> "$OUT/${c}_shard.err" || { tail -30 "$OUT/${c}_shard.err"; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/${c}_shard.json')); print('$c shard', d['ms_per_step'], d['config'].get('single_pass_ms'), d.get('kernel_ms'), d['roofline']['kernel'])"
  done
fi
if has prof; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o bench -- \
      python3 bench.py --no-cpu --no-e2e --inflight 1 > "$OUT/c4_bench_under_rocprof.json" 2> "$OUT/prof.err" || { tail -30 "$OUT/prof.err"; exit 1; }
  find "$OUT/prof" -name "*kernel_stats.csv" | head -3
fi
if has configs; then
  for c in ${CONFIGS:-c2 c3 c5}; do
    timeout -k 10 300 python3 bench.py --config $c --no-e2e > "$OUT/${c}_bench.json" 2> "$OUT/${c}_bench.err" || { tail -30 "$OUT/${c}_bench.err"; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/${c}_bench.json')); print('$c', d['value'], d['ms_per_step'], d['config'].get('single_pass_ms'), d['roofline']['kernel'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$c" -o bench -- \
        python3 bench.py --config $c --no-cpu --no-e2e --inflight 1 > "$OUT/${c}_under_rocprof.json" 2> "$OUT/prof_$c.err" || { tail -30 "$OUT/prof_$c.err"; exit 1; }
  done
fi
exit 0
