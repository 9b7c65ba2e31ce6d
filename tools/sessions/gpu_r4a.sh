#!/bin/bash
# round 4 baseline: single-sample shard rehearsals (C5 1/8 and 7/8, C5 whole, C4 1/8) and the
# rocprof kernel summary of the C5 1/8 shard
OUT=gpurun_out/r4a
mkdir -p $OUT
export TMPDIR=/tmp
for s in 0/8 7/8 0/1; do
  CFG=c5 timeout -k 10 300 python3 tools/diag_shard_kernels.py $s auto >> $OUT/shard.log 2>&1 || { tail $OUT/shard.log; exit 1; }
done
CFG=c4 timeout -k 10 300 python3 tools/diag_shard_kernels.py 0/8 auto >> $OUT/shard.log 2>&1 || { tail $OUT/shard.log; exit 1; }
grep ms/pass $OUT/shard.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof5 -o p -- python3 bench.py --config c5 --sim-shard 0/8 --no-cpu --no-e2e --inflight 1 > $OUT/c5s.json 2> $OUT/c5s.err || { tail $OUT/c5s.err; exit 1; }
cut -d, -f1-4 $OUT/prof5/p_kernel_stats.csv | head -12
