#!/bin/bash
# PMC SQ passes of the C4 pass (locate / heavy / lean pileup counters)
OUT=gpurun_out/r3g
mkdir -p $OUT
export TMPDIR=/tmp
PASSES=sq bash tools/pmc.sh $OUT/pmc c4
python3 tools/pmc_kernels.py $OUT/pmc rcp_locate rcp_heavy rcp_pileup_lean > $OUT/sq_c4.txt; cat $OUT/sq_c4.txt
