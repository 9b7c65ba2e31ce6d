#!/bin/bash
# fused edge pass for uniform non-power-of-two bins (scan_bins_uni): GPU suite on the in-tree
# library, then A/B old (-DRCP_NO_UNI_BINS=1) / new on C2 (D = 1 and auto, two reps) and C4
OUT=gpurun_out/r3f3
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
for rep in 1 2; do
for v in old new; do
  lib=build_var/$v/librecoup_amd.so
  for d in 1 auto; do
    RCP_LIB_PATH=$lib timeout -k 10 200 python3 bench.py --config c2 --no-e2e --inflight $d --steps 20 > $OUT/${v}_c2_$d.json 2> $OUT/${v}_c2_$d.err || { tail $OUT/${v}_c2_$d.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/${v}_c2_$d.json')); print('$v c2 D=$d', round(d['ms_per_step'],4), 'single', round(d['config']['single_pass_ms'],4), {k: round(x,4) for k,x in d['kernel_ms'].items()}, 'frac', round(d['roofline']['frac'],3), 'parity', d.get('parity_sample'))" | tee -a $OUT/ab.log
  done
done
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o c2 -- python3 bench.py --config c2 --no-cpu --no-e2e --inflight 1 > $OUT/c2_rocprof_bench.json 2> $OUT/c2_prof.err || { tail $OUT/c2_prof.err; exit 1; }
grep -E "pileup|locate|heavy" $OUT/prof/c2_kernel_stats.csv | cut -d, -f1-5
