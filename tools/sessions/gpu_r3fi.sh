#!/bin/bash
# interpolated rows as the first blocks of the row-wave grid: GPU suite, C3 A/B
OUT=gpurun_out/r3fi
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
BENCH_ARGS="--inflight 1" bash tools/gpu_ab.sh $OUT c3 base nofuse base nofuse base nofuse || exit 1
bash tools/gpu_ab.sh $OUT c3 base nofuse || exit 1
