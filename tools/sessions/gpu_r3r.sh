#!/bin/bash
# (1) Rle run counts fused into the coverage pileup: parity tests + C4 rle-path kernel stats;
# (2) which pileup kernel serves a small shard best: 1/8, 1/4 and all of C4 on lean (auto),
# row-wave (rows), general
OUT=gpurun_out/r3r
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_rle.py \
  tests/test_gpu_abi.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
ITERS=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c4 -o p -- python3 tools/prof_rle.py c4 \
  > $OUT/prof_rle_c4.log 2>&1 || { tail -20 $OUT/prof_rle_c4.log; exit 1; }
grep -E "iter|equal" $OUT/prof_rle_c4.log
grep -E "pileup_kernel<false, true>|seams|emit|count" $OUT/prof_c4/p_kernel_stats.csv
for s in 0/8 0/6 0/5 0/4; do
timeout -k 10 300 python3 tools/diag_shard_kernels.py $s auto general >> $OUT/kernels.log 2> $OUT/kernels.err || { tail $OUT/kernels.err; exit 1; }
done
cat $OUT/kernels.log
