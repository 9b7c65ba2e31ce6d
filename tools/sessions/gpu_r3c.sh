#!/bin/bash
# RLE tile kernel with dense windows: RLE GPU tests, then occupancy A/B (8 vs 4 waves/SIMD) under rocprof
OUT=gpurun_out/r3c
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_rle.py tests/test_gpu_rshim.py tests/test_gpu_abi.py tests/test_gpu_api.py -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
for v in wpe8 wpe4 wpe8; do
  RCP_LIB_PATH=build_var/$v/librecoup_amd.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$v -o rle -- python3 tools/prof_rle.py c4 > $OUT/prof_rle_$v.log 2>&1 || { tail $OUT/prof_rle_$v.log; exit 1; }
  echo $v; grep -E "iter 2|equal" $OUT/prof_rle_$v.log
  grep -E "rle_tile|rle_emit|rle_count|pileup_kernel<false, true>" $OUT/prof_$v/rle_kernel_stats.csv | cut -d, -f1-4
done
