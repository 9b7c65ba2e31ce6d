#!/bin/bash
# RLE path v2 end of milestone: all GPU tests, bench lines with the rle_path leg (C4, C2), PMC traffic of the RLE kernels (C4)
OUT=gpurun_out/r3e
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 400 python bench.py > $OUT/c4_bench.json 2> $OUT/c4_bench.err || { tail $OUT/c4_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/c4_bench.json')); print('c4', d['value'], d['ms_per_step'], d['roofline']['frac'], d['e2e']['ms'], d['e2e']['rle_path'])"
timeout -k 10 400 python bench.py --config c2 > $OUT/c2_bench.json 2> $OUT/c2_bench.err || { tail $OUT/c2_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/c2_bench.json')); print('c2', d['value'], d['ms_per_step'], d['roofline']['frac'], d['e2e']['ms'], d['e2e']['rle_path'])"
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d $OUT/pmc_$ctr -o p -- python3 tools/prof_rle.py c4 > $OUT/pmc_$ctr.log 2>&1 || { tail $OUT/pmc_$ctr.log; exit 1; }
done
python3 tools/pmc_kernels.py $OUT rle_ pileup_kernel > $OUT/pmc_rle_c4.txt; cat $OUT/pmc_rle_c4.txt
