#!/bin/bash
# 1/8 and 1/6 C4 shards after the start-only stream: lean (forced) vs auto (general below 36k rows)
OUT=gpurun_out/r3s2
mkdir -p $OUT
export TMPDIR=/tmp
for s in 0/8 0/6; do
timeout -k 10 300 python3 tools/diag_shard_kernels.py $s auto lean >> $OUT/kernels.log 2> $OUT/kernels.err || { tail $OUT/kernels.err; exit 1; }
done
cat $OUT/kernels.log
