#!/bin/bash
OUT=gpurun_out/r02y
mkdir -p $OUT
export TMPDIR=/tmp
PASSES=sq timeout -k 10 500 bash tools/pmc.sh $OUT/sq_c3 c3 || { echo "sq c3 failed"; exit 1; }
python3 tools/pmc_sum.py -k rcp_ $OUT/sq_c3
