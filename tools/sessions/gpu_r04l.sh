#!/bin/bash
# A/B: merged-layout chunk ranges as dense (row, chunk) words (dense) vs stream 0 of three (base)
OUT=gpurun_out/r04l
mkdir -p $OUT
export TMPDIR=/tmp
RCP_LIB_PATH=build_var/dense/librecoup_amd.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/dense_tests.log 2>&1 || { tail -30 $OUT/dense_tests.log; exit 1; }
tail -1 $OUT/dense_tests.log
BENCH_ARGS="--inflight 1" bash tools/gpu_ab.sh $OUT "c4 c5 c2" base dense base dense
