#!/bin/bash
# A/B: edge-position reads counted per pair (one LDS add per piece edge) vs per-read atomics
OUT=gpurun_out/r04e
mkdir -p $OUT
export TMPDIR=/tmp
RCP_LIB_PATH=build_var/edge/librecoup_amd.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/edge_tests.log 2>&1 || { tail -30 $OUT/edge_tests.log; exit 1; }
tail -1 $OUT/edge_tests.log
bash tools/gpu_ab.sh $OUT c3 base edge base edge
