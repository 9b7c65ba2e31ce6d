#!/bin/bash
# end-of-session check of the committed tree: GPU tests, smoke, default bench line, config lines
OUT=gpurun_out/r03d
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail $OUT/smoke.log; exit 1; }
for c in c4 c3 c5 c2; do
  timeout -k 10 600 python3 bench.py --config $c > $OUT/${c}_bench.json 2> $OUT/${c}_bench.err || { tail $OUT/${c}_bench.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/${c}_bench.json')); print('$c', round(d['ms_per_step'],4), '%.3e' % d['value'], d['config']['inflight'], d['config']['inflight_note'][-48:], {k: round(x,4) for k,x in d['kernel_ms'].items()}, round(d['roofline']['frac'],3), d['parity_sample'], round(d['e2e']['ms'],1))"
done
for sh in 0/8 7/8; do
  timeout -k 10 300 python bench.py --no-cpu --no-e2e --sim-shard $sh > $OUT/shard_${sh/\//of}.json 2> $OUT/shard_${sh/\//of}.err || { tail $OUT/shard_${sh/\//of}.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/shard_${sh/\//of}.json')); print('$sh', round(d['ms_per_step'],4), d['config']['inflight'], d['config']['inflight_note'][-48:])"
done
