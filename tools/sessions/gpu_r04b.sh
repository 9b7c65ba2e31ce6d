#!/bin/bash
# A/B: row-wave kernel windows piped across parts (RCP_RW_PIPE) vs base; parity of the variant first
OUT=gpurun_out/r04b
mkdir -p $OUT
export TMPDIR=/tmp
RCP_LIB_PATH=build_var/pipe/librecoup_amd.so timeout -k 10 300 python -u -m pytest tests/test_gpu_rows.py tests/test_gpu_c3.py tests/test_gpu_configs.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pipe_tests.log 2>&1 || { tail -30 $OUT/pipe_tests.log; exit 1; }
tail -1 $OUT/pipe_tests.log
bash tools/gpu_ab.sh $OUT c3 base pipe base pipe
