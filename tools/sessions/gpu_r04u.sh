#!/bin/bash
# A/B: passes in flight with each lean launch confined to one XCD half (xsplit: launches alternate
# halves) vs every launch on all XCDs (base); the bench picks D = 1..3 by timing either way
OUT=gpurun_out/r04u
mkdir -p $OUT
export TMPDIR=/tmp
RCP_LIB_PATH=build_var/xsplit/librecoup_amd.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/xsplit_tests.log 2>&1 || { tail -30 $OUT/xsplit_tests.log; exit 1; }
tail -1 $OUT/xsplit_tests.log
for v in base xsplit base xsplit; do
  for c in c4 c5; do
    RCP_LIB_PATH=build_var/$v/librecoup_amd.so timeout -k 10 300 python3 bench.py --config $c --no-cpu --no-e2e > $OUT/${v}_$c.json 2> $OUT/${v}_$c.err || { tail $OUT/${v}_$c.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/${v}_$c.json')); print('$v $c', round(d['ms_per_step'],4), d['config']['inflight'], d['config']['inflight_note'][-50:])" | tee -a $OUT/ab.log
  done
done
