#!/bin/bash
# A/B: per-pair orientation as a uniform branch in the pair add loop (urev) vs a select per read (base)
OUT=gpurun_out/r04h
mkdir -p $OUT
export TMPDIR=/tmp
RCP_LIB_PATH=build_var/urev/librecoup_amd.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/urev_tests.log 2>&1 || { tail -30 $OUT/urev_tests.log; exit 1; }
tail -1 $OUT/urev_tests.log
bash tools/gpu_ab.sh $OUT c3 base urev base urev
