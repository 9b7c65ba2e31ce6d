#!/bin/bash
# end-of-session check of the committed tree: GPU tests, smoke, every config's bench line (CPU
# baseline and e2e included), rocprof kernel stats of the C4 bench, PMC traffic of the C4 pileup,
# the 1/8 shard rehearsals
OUT=gpurun_out/r04j
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
for c in c4 c3 c5 c2; do
  timeout -k 10 600 python3 bench.py --config $c > $OUT/${c}_bench.json 2> $OUT/${c}_bench.log || { tail $OUT/${c}_bench.log; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/${c}_bench.json')); print('$c', round(d['ms_per_step'],4), '%.3e' % d['value'], d['config']['inflight'], {k: round(x,4) for k,x in d['kernel_ms'].items()}, round(d['roofline']['frac'],3), d['roofline']['traffic'], d['parity_sample'], round(d['e2e']['ms'],1), '%.3e' % d['cpu_baseline']['value'])"
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/rocprof_c4 -o bench -- \
    python3 bench.py --no-cpu --no-e2e --inflight 1 > $OUT/c4_bench_under_rocprof.json 2> $OUT/rocprof_c4.err || { tail $OUT/rocprof_c4.err; exit 1; }
for sh in 0/8 7/8; do
  timeout -k 10 300 python bench.py --no-cpu --no-e2e --sim-shard $sh > $OUT/shard_${sh/\//of}.json 2> $OUT/shard_${sh/\//of}.log || { tail $OUT/shard_${sh/\//of}.log; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/shard_${sh/\//of}.json')); print('$sh', round(d['ms_per_step'],4), d['config']['inflight'])"
done
