#!/bin/bash
# PMC traffic (FETCH_SIZE / WRITE_SIZE, separate passes) of the pileup kernel for every config after
# the dense chunk-range change, then the calibrated per-launch bytes (profiles/traffic_<config>.json)
OUT=gpurun_out/r04m
mkdir -p $OUT
export TMPDIR=/tmp
for c in c4 c5 c2 c3; do
  PASSES=traffic timeout -k 10 500 bash tools/pmc.sh $OUT/pmc_$c $c || { echo "pmc $c failed"; tail $OUT/pmc_$c/*.log; exit 1; }
  python3 tools/pmc_traffic.py $OUT/pmc_$c $OUT/traffic_$c.json profiles/fetch_calib.json || exit 1
  python3 -c "import json; d=json.load(open('$OUT/traffic_$c.json')); print('$c', d['kernel'], round(d['hbm_bytes_per_launch']/1e9, 4), 'GB', d['dispatches'])"
done
