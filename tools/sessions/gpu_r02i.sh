#!/bin/bash
OUT=gpurun_out/r02i
mkdir -p $OUT
export TMPDIR=/tmp
RCP_LIB_PATH=build_var/timing/librecoup_amd.so timeout -k 10 300 python3 tools/diag_e2e.py c4 > $OUT/diag_e2e_timing.log 2>&1 || { tail $OUT/diag_e2e_timing.log; exit 1; }
cat $OUT/diag_e2e_timing.log | head -120
