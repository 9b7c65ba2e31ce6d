#!/bin/bash
# SQ counters of the C4 step's kernels (locate / heavy / reset), PMC traffic of the C3 row-wave kernel
OUT=gpurun_out/r02f
mkdir -p $OUT
export TMPDIR=/tmp
PASSES=sq timeout -k 10 500 bash tools/pmc.sh $OUT/sq_c4 c4 || { echo "sq c4 failed"; exit 1; }
python3 tools/pmc_sum.py -k rcp_ $OUT/sq_c4
PASSES=traffic timeout -k 10 400 bash tools/pmc.sh $OUT/pmc_c3 c3 || { echo "pmc c3 failed"; exit 1; }
python3 tools/pmc_traffic.py $OUT/pmc_c3 $OUT/traffic_c3.json profiles/fetch_calib.json
cat $OUT/traffic_c3.json
