#!/bin/bash
OUT=gpurun_out/r02c
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo TESTS FAILED; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 300 python3 tools/diag_e2e.py c4 2>&1 | grep -v amdgpu.ids > $OUT/diag_e2e_c4.log; cat $OUT/diag_e2e_c4.log
for k in 0/2 0/4 0/8 3/8 7/8; do
  n=${k/\//of}
  timeout -k 10 300 python3 bench.py --sim-shard $k --no-cpu --no-e2e > $OUT/shard_$n.json 2> $OUT/shard_$n.err || { tail $OUT/shard_$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/shard_$n.json')); print('shard $k', d['config']['rank0_shard']['regions'], round(d['ms_per_step'],4), {k: round(v,4) for k,v in d['kernel_ms'].items()}, round(d['roofline']['frac'],3))"
done
for c in c4 c5 c2 c3; do
  timeout -k 10 600 python3 bench.py --config $c > $OUT/${c}_bench.json 2> $OUT/${c}_bench.err || { tail $OUT/${c}_bench.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/${c}_bench.json')); print('$c', round(d['ms_per_step'],4), '%.3g' % d['value'], {k: round(v,4) for k,v in d['kernel_ms'].items()}, 'frac', round(d['roofline']['frac'],3), 'step', round(d['roofline']['step_frac'],3), 'e2e', round(d['e2e']['ms'],1), d['e2e']['phases_ms'], 'cpu', '%.3g' % d['cpu_baseline']['value'], d['parity_sample'])"
done
