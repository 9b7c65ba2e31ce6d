#!/bin/bash
# strand codes 2 bits per read over PCIe: GPU suite on the in-tree library, then e2e A/B
# old (-DRCP_NO_STRAND2=1) / new on C5 and C4 (bench e2e legs, two reps)
OUT=gpurun_out/${OUTD:-r3f4}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu ${TESTS:-tests} > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
for rep in 1 2; do
for c in ${CFGS:-c5 c4}; do
for v in old new; do
  lib=build_var/$v/librecoup_amd.so
  RCP_LIB_PATH=$lib timeout -k 10 300 python3 bench.py --config $c --no-cpu --inflight 1 --steps 5 > $OUT/${v}_$c.json 2> $OUT/${v}_$c.err || { tail $OUT/${v}_$c.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/${v}_$c.json')); e=d['e2e']
print('$v $c e2e', round(e['ms'],1), {k: round(x,1) for k,x in e['phases_ms'].items()}, 'calls', e['calls_ms'], 'any', round(e['any_order']['ms'],1), {k: round(x,1) for k,x in e['any_order']['phases_ms'].items()}, 'parity', (d.get('parity_sample') or {}).get('ok'))" | tee -a $OUT/ab.log
done
done
done
