#!/bin/bash
OUT=gpurun_out/r02m
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python tools/diag_overlap.py c4 20 > $OUT/overlap_c4.log 2>&1 || { tail -5 $OUT/overlap_c4.log; exit 1; }
for sh in 0/8 0/4 0/2; do
timeout -k 10 300 python tools/diag_overlap.py c4 40 $sh > $OUT/overlap_c4_s${sh/\//of}.log 2>&1 || { tail -5 $OUT/overlap_c4_s${sh/\//of}.log; exit 1; }
done
timeout -k 10 300 python tools/diag_overlap.py c5 20 > $OUT/overlap_c5.log 2>&1 || { tail -5 $OUT/overlap_c5.log; exit 1; }
grep -h "^c" $OUT/overlap_*.log
