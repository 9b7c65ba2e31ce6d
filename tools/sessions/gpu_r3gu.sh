#!/bin/bash
# start-only stream in the general kernel too: GPU suite, then same-box A/B (base vs no start-only
# stream) on C2, the 1/8 C4 shard and the C4 Rle path (coverage pileup)
OUT=gpurun_out/r3gu
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
BENCH_ARGS="--inflight 1" bash tools/gpu_ab.sh $OUT "c2 c5" base nouni base nouni || exit 1
BENCH_ARGS="--inflight 1 --sim-shard 0/8" TAG=_s8 bash tools/gpu_ab.sh $OUT c4 base nouni base nouni || exit 1
for v in base nouni; do
RCP_LIB_PATH=build_var/$v/librecoup_amd.so ITERS=3 timeout -k 10 300 python3 tools/prof_rle.py c4 > $OUT/rle_$v.log 2>&1 || { tail $OUT/rle_$v.log; exit 1; }
echo "$v"; grep -E "iter|equal" $OUT/rle_$v.log
done
