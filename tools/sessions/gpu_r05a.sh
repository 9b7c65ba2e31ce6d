#!/bin/bash
# A/B: lean kernel reads as 16-B pairs of consecutive reads (x4) vs 8-B reads 64 apart (base)
OUT=gpurun_out/r05a
mkdir -p $OUT
export TMPDIR=/tmp
RCP_LIB_PATH=build_var/x4/librecoup_amd.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/x4_tests.log 2>&1 || { tail -30 $OUT/x4_tests.log; exit 1; }
tail -1 $OUT/x4_tests.log
BENCH_ARGS="--inflight 1" bash tools/gpu_ab.sh $OUT "c4 c5" base x4 base x4 base x4
