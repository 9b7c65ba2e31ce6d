#!/bin/bash
OUT=gpurun_out/r02l
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 python tools/dbg_lean_rounds.py > $OUT/dbg.log 2>&1 || { tail -5 $OUT/dbg.log; exit 1; }
cat $OUT/dbg.log | grep -v amdgpu.ids
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
for sh in 0/8 7/8 0/4 0/2; do
  BENCH_ARGS="--sim-shard $sh" TAG="_s${sh/\//of}" bash tools/gpu_ab.sh $OUT "c4" r4 base r4 base || exit 1
done
bash tools/gpu_ab.sh $OUT "c4 c5" r4 base || exit 1
