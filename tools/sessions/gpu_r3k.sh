#!/bin/bash
# A/B heavy slice grid 4096 / 1024 / 512 / 256 blocks (C4 has 321 heavy rows; C5 / 1/8 shard none or few); pool tests
OUT=gpurun_out/r3k
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_abi.py tests/test_gpu_lean.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
BENCH_ARGS="--inflight 1" bash tools/gpu_ab.sh $OUT "c4 c5" g4096 g1024 g512 g256 g4096 g1024 g512 g256 || exit 1
BENCH_ARGS="--inflight 1 --sim-shard 0/8" TAG=_s8 bash tools/gpu_ab.sh $OUT "c4" g4096 g1024 g512 g256 || exit 1
