#!/bin/bash
# readsets built entirely from the device pool: C5 repeated builds, GPU tests, C5 / C4 e2e
OUT=gpurun_out/r04s
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python tools/diag_readset.py c5 10 > $OUT/readset_c5.log 2>&1 || { tail $OUT/readset_c5.log; exit 1; }
grep -v amdgpu.ids $OUT/readset_c5.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/t.log 2>&1 || { tail -30 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
for c in c5 c4; do
  timeout -k 10 600 python3 bench.py --config $c --no-cpu > $OUT/${c}_bench.json 2> $OUT/${c}_bench.log || { tail $OUT/${c}_bench.log; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/${c}_bench.json')); e=d['e2e']; print('$c', round(d['ms_per_step'],4), 'e2e', round(e['ms'],1), e['calls_ms'], e['width_runs'], 'any', e['any_order']['calls_ms'])"
done
