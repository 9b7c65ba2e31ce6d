#!/bin/bash
OUT=gpurun_out/r02h
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
bash tools/gpu_ab.sh $OUT "c4" prev base prev base || exit 1
bash tools/gpu_ab.sh $OUT "c3" base ring3 base ring3 || exit 1
bash tools/gpu_ab.sh $OUT "c2 c5" prev base || exit 1
