#!/bin/bash
# interleaved candidate slots in the pair streams (C3 row-wave kernel): parity then A/B
OUT=gpurun_out/r3il
mkdir -p $OUT
export TMPDIR=/tmp
RCP_LIB_PATH=build_var/inter/librecoup_amd.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_rows.py tests/test_gpu_lean.py tests/test_gpu_random.py tests/test_gpu_configs.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
BENCH_ARGS="--inflight 1" bash tools/gpu_ab.sh $OUT c3 base inter base inter base inter || exit 1
