#!/bin/bash
# C3 row-wave kernel counters after the folded-offset adds: SQ passes + traffic
OUT=gpurun_out/r3c3
mkdir -p $OUT
export TMPDIR=/tmp
PASSES=sq bash tools/pmc.sh $OUT/pmc c3 || exit 1
PASSES=traffic bash tools/pmc.sh $OUT/pmc c3 || exit 1
python3 tools/pmc_kernels.py $OUT/pmc rows_kernel interp
