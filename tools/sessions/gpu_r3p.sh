#!/bin/bash
# Stranded layout built at first use for host-uploaded readsets: GPU tests, e2e of C4 / C5
OUT=gpurun_out/r3p
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
for c in c4 c5; do
timeout -k 10 400 python bench.py --config $c --no-cpu --steps 10 > $OUT/${c}_bench.json 2> $OUT/${c}_bench.err || { tail $OUT/${c}_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/${c}_bench.json')); e=d['e2e']; print('$c', round(d['ms_per_step'],4), 'e2e', round(e['ms'],1), {k: round(v,1) for k,v in e['phases_ms'].items()}, e['calls_ms'], 'any', round(e['any_order']['ms'],1), {k: round(v,1) for k,v in e['any_order']['phases_ms'].items()}, 'rle', round(e['rle_path']['ms'],1), e['rle_path']['equal_fused'])"
done
