#!/bin/bash
# round 4: general kernel rounds per workgroup on the C4 1/8 shard: 1 (g1) / 2 (new) / 4 (g4)
OUT=gpurun_out/r4zb
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
  for v in new g1 g4; do
    lib=build_var/$v/librecoup_amd.so
    [ $v = new ] && lib=recoup_amd/librecoup_amd.so
    echo "== $v" >> $OUT/ab.log
    RCP_LIB_PATH=$lib CFG=c4 timeout -k 10 200 python3 tools/diag_shard_kernels.py 0/8 auto general >> $OUT/ab.log 2>&1 || { tail $OUT/ab.log; exit 1; }
  done
done
grep -E "==|ms/pass" $OUT/ab.log
