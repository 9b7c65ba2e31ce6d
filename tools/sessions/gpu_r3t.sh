#!/bin/bash
# full GPU suite + smoke after the fused Rle counts and the small-table kernel rule; the 1/8
# and 1/4 C4 shard rehearsals (D auto) and the N=1 bench
OUT=gpurun_out/r3t
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
for s in 0/8 7/8 0/4; do
n=$(echo $s | tr / o)
timeout -k 10 300 python3 bench.py --sim-shard $s --no-cpu --no-e2e > $OUT/shard_$n.json 2> $OUT/shard_$n.err || { tail $OUT/shard_$n.err; exit 1; }
python3 -c "import json,sys; d=json.load(open('$OUT/shard_$n.json')); print('$s', d['ms_per_step'], d.get('inflight_note'))"
done
timeout -k 10 600 python3 bench.py --no-cpu > $OUT/c4_bench.json 2> $OUT/c4_bench.err || { tail $OUT/c4_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/c4_bench.json')); print('c4', d['value'], d['ms_per_step'], d.get('inflight_note'), d['roofline']['frac'])"
