#!/bin/bash
# lean work items of two rounds (32 rows) vs four (64) vs the general kernel; parity of the
# two-round items first (lean tests + C4 reduced, bit-equal to the general kernel)
OUT=gpurun_out/r3v
mkdir -p $OUT
export TMPDIR=/tmp
for v in l2 g2; do
RCP_LIB_PATH=build_var/$v/librecoup_amd.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_lean.py tests/test_gpu_configs.py tests/test_gpu_random.py --deselect tests/test_gpu_lean.py::test_lean_kernel_choice > $OUT/tests_$v.log 2>&1 || { tail -30 $OUT/tests_$v.log; exit 1; }
tail -1 $OUT/tests_$v.log
done
export BENCH_ARGS="--inflight 1"
bash tools/gpu_ab.sh $OUT c2 base g4 g2 || exit 1
bash tools/gpu_ab.sh $OUT "c4 c5" base l4 l2 || exit 1
BENCH_ARGS="--inflight 1 --sim-shard 0/8" TAG=_s8 bash tools/gpu_ab.sh $OUT "c4 c5" base l4 l2 || exit 1
BENCH_ARGS="--inflight 1 --sim-shard 0/4" TAG=_s4 bash tools/gpu_ab.sh $OUT "c4 c5" base l4 l2 || exit 1
