#!/bin/bash
# A/B: row-wave kernel: record + row-info loads hoisted (hoist), windows piped without the per-part fallback (pipe2)
OUT=gpurun_out/r04c
mkdir -p $OUT
export TMPDIR=/tmp
RCP_LIB_PATH=build_var/hoist/librecoup_amd.so timeout -k 10 300 python -u -m pytest tests/test_gpu_rows.py tests/test_gpu_c3.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/hoist_tests.log 2>&1 || { tail -30 $OUT/hoist_tests.log; exit 1; }
tail -1 $OUT/hoist_tests.log
bash tools/gpu_ab.sh $OUT c3 base hoist pipe2 base hoist pipe2
