#!/bin/bash
# RLE tile kernel: dense / generic split, branch-free batch loads with deferred start subtraction
OUT=gpurun_out/r3d
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_rle.py tests/test_gpu_rshim.py tests/test_gpu_abi.py tests/test_gpu_api.py tests/test_gpu_c1.py -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
for c in c4 c5 c2 c3; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$c -o rle -- python3 tools/prof_rle.py $c > $OUT/prof_rle_$c.log 2>&1 || { tail $OUT/prof_rle_$c.log; exit 1; }
echo $c; grep -E "iter 2|equal" $OUT/prof_rle_$c.log
grep -E "rle_tile|rle_interp|rle_emit|rle_count|pileup_kernel<false, true>" $OUT/prof_$c/rle_kernel_stats.csv | cut -d, -f1-4
done
