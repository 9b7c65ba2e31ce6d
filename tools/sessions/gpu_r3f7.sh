#!/bin/bash
# SQ counters of C2's kernels (general pileup, locate, heavy): where the general kernel's
# skeleton time goes (next round's C2 work)
OUT=gpurun_out/r3f7
mkdir -p $OUT
export TMPDIR=/tmp
PASSES=sq bash tools/pmc.sh $OUT/pmc c2 || { tail $OUT/pmc/*.log; exit 1; }
python3 tools/pmc_kernels.py $OUT/pmc pileup locate heavy > $OUT/c2_sq.txt 2>&1
cat $OUT/c2_sq.txt
