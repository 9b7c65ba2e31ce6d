#!/bin/bash
# round 4: lean kernel with 10 pile waves (lp10, 7 waves / SIMD) vs 8 (new)
OUT=gpurun_out/r4za
mkdir -p $OUT
export TMPDIR=/tmp
T="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread"
RCP_LIB_PATH=build_var/lp10/librecoup_amd.so timeout -k 10 300 $T -m gpu tests/test_gpu_lean.py tests/test_gpu_random.py > $OUT/lean_lp10.log 2>&1 || { tail -30 $OUT/lean_lp10.log; exit 1; }
echo "lp10 $(tail -1 $OUT/lean_lp10.log)"
for rep in 1 2; do
  for v in new lp10; do
    lib=build_var/$v/librecoup_amd.so
    [ $v = new ] && lib=recoup_amd/librecoup_amd.so
    for c in c4 c5; do
      RCP_LIB_PATH=$lib timeout -k 10 300 python3 bench.py --config $c --no-cpu --no-e2e > $OUT/${v}_${c}_$rep.json 2> $OUT/${v}_${c}_$rep.err || { tail $OUT/${v}_${c}_$rep.err; exit 1; }
      python3 -c "
import json; d=json.load(open('$OUT/${v}_${c}_$rep.json')); c=d['config']
print('$v $c', round(d['ms_per_step'],4), c['inflight_note'].split('by D: ')[-1], 'kern', round(d['roofline']['kernel_ms'],4), d['inflight_check']['equal_to_general_kernel'])"
    done
  done
done
