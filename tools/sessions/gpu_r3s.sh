#!/bin/bash
# small-shard kernel choice on C5 too, and the per-kernel times of one 1/8 C4 shard pass
OUT=gpurun_out/r3s
mkdir -p $OUT
export TMPDIR=/tmp
for s in 0/8 0/4; do
CFG=c5 timeout -k 10 300 python3 tools/diag_shard_kernels.py $s auto general >> $OUT/kernels.log 2> $OUT/kernels.err || { tail $OUT/kernels.err; exit 1; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_s8 -o p -- python3 tools/diag_shard_kernels.py 0/8 auto general \
  > $OUT/prof_s8.log 2>&1 || { tail -20 $OUT/prof_s8.log; exit 1; }
cat $OUT/kernels.log
cut -c1-150 $OUT/prof_s8/p_kernel_stats.csv | head -14
