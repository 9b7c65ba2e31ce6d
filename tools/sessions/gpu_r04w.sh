#!/bin/bash
# A/B: row-wave kernel occupancy -- 1023-position windows (LDS per wave halved) at 4 / 5 / 6 waves
# per SIMD (the last two with VGPR spills) vs 2047-position windows at 4
OUT=gpurun_out/r04w
mkdir -p $OUT
export TMPDIR=/tmp
for v in sh4w5 sh4w6; do
  RCP_LIB_PATH=build_var/$v/librecoup_amd.so timeout -k 10 300 python -u -m pytest tests/test_gpu_rows.py tests/test_gpu_c3.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/${v}_tests.log 2>&1 || { tail -30 $OUT/${v}_tests.log; exit 1; }
  tail -1 $OUT/${v}_tests.log
done
BENCH_ARGS="--inflight 1" bash tools/gpu_ab.sh $OUT c3 base sh4 sh4w5 sh4w6 base sh4 sh4w5 sh4w6
