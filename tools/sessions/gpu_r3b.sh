#!/bin/bash
# RLE path v2 (tile kernel, count/emit encode, device-resident coverage handle): GPU tests, R-path timing
OUT=gpurun_out/r3b
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_rle -o rle -- python3 tools/prof_rle.py c4 > $OUT/prof_rle_c4.log 2>&1 || { tail $OUT/prof_rle_c4.log; exit 1; }
grep -E "iter|equal" $OUT/prof_rle_c4.log
for c in c2 c3 c5; do
  timeout -k 10 300 python3 tools/prof_rle.py $c > $OUT/rle_$c.log 2>&1 || { tail $OUT/rle_$c.log; exit 1; }
  echo $c; grep -E "iter|equal" $OUT/rle_$c.log
done
