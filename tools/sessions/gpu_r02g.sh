#!/bin/bash
# Reset folded into locate: GPU tests; locate variants A/B (C4, C2, C5); C3 row-wave PMC traffic
OUT=gpurun_out/r02g
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
for c in c4 c2 c5; do
  for v in base wpe8 cedir cedir8 base; do
    RCP_LIB_PATH=build_var/$v/librecoup_amd.so timeout -k 10 200 python3 bench.py --config $c --no-cpu --no-e2e --steps 30 > $OUT/${v}_$c.json 2> $OUT/${v}_$c.err || { tail $OUT/${v}_$c.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/${v}_$c.json')); print('$v $c', round(d['ms_per_step'],4), {k: round(x,4) for k,x in d['kernel_ms'].items()}, d['parity_sample'])"
  done
done
PASSES=traffic timeout -k 10 400 bash tools/pmc.sh $OUT/pmc_c3 c3 || { echo "pmc c3 failed"; exit 1; }
python3 tools/pmc_traffic.py $OUT/pmc_c3 $OUT/traffic_c3.json profiles/fetch_calib.json
cat $OUT/traffic_c3.json
