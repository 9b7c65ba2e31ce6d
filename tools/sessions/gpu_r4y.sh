#!/bin/bash
# round 4 end check: full GPU suite + smoke on the committed tree, C4 default bench line
OUT=gpurun_out/r4y
mkdir -p $OUT
export TMPDIR=/tmp
T="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 600 $T -m gpu tests > $OUT/tests.log 2>&1 || { tail -60 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -30 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python3 bench.py > $OUT/c4.json 2> $OUT/c4.err || { tail $OUT/c4.err; exit 1; }
cat $OUT/c4.json
