#!/bin/bash
# RLE profile: run starts from the lengths (no device scan) when slices start at position 0
OUT=gpurun_out/r3l
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_rle.py tests/test_gpu_rshim.py tests/test_gpu_abi.py tests/test_gpu_api.py tests/test_gpu_c1.py -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
for c in c4 c5 c3; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$c -o rle -- python3 tools/prof_rle.py $c > $OUT/prof_rle_$c.log 2>&1 || { tail $OUT/prof_rle_$c.log; exit 1; }
echo $c; grep -E "iter 2|equal" $OUT/prof_rle_$c.log
python3 tools/kstat_rle.py $OUT/prof_$c/rle_kernel_stats.csv
done
