#!/bin/bash
# uniform-width layouts skip the segmented pmax scan: GPU suite, readset phase times (timing
# build), C5 / C4 e2e
OUT=gpurun_out/r3pm
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
RCP_LIB_PATH=build_var/tim/librecoup_amd.so timeout -k 10 300 python3 tools/diag_readset.py c5 3 > $OUT/readset_c5.log 2>&1 || { tail $OUT/readset_c5.log; exit 1; }
grep -E "rep|plan\]" $OUT/readset_c5.log | tail -12
for c in c5 c4; do
timeout -k 10 600 python3 bench.py --config $c --no-cpu --steps 10 > $OUT/$c.json 2> $OUT/$c.err || { tail $OUT/$c.err; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/$c.json')); e=d['e2e']
print('$c', round(d['ms_per_step'],4), 'e2e', round(e['ms'],1), {k: round(v,1) for k,v in e['phases_ms'].items()}, 'any', round(e['any_order']['ms'],1), 'rle', round(e['rle_path']['ms'],1))"
done
