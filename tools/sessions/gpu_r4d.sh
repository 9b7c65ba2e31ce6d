#!/bin/bash
# round 4: ablations of the lean kernel on the C5 1/8 shard and of the general kernel on C2 / the C4 1/8 shard;
# C2 on the general / row-wave / lean-any kernels
OUT=gpurun_out/r4d
mkdir -p $OUT
export TMPDIR=/tmp
for v in base abl1 abl2 abl3; do
  echo "== $v" >> $OUT/ab.log
  RCP_LIB_PATH=build_var/$v/librecoup_amd.so CFG=c5 timeout -k 10 200 python3 tools/diag_shard_kernels.py 0/8 auto >> $OUT/ab.log 2>&1 || { tail $OUT/ab.log; exit 1; }
done
for v in base gabl1 gabl2 gabl3; do
  echo "== $v" >> $OUT/ab.log
  RCP_LIB_PATH=build_var/$v/librecoup_amd.so CFG=c2 timeout -k 10 200 python3 tools/diag_shard_kernels.py 0/1 general >> $OUT/ab.log 2>&1 || { tail $OUT/ab.log; exit 1; }
  RCP_LIB_PATH=build_var/$v/librecoup_amd.so CFG=c4 timeout -k 10 200 python3 tools/diag_shard_kernels.py 0/8 general >> $OUT/ab.log 2>&1 || { tail $OUT/ab.log; exit 1; }
done
echo "== kernels" >> $OUT/ab.log
CFG=c2 timeout -k 10 200 python3 tools/diag_shard_kernels.py 0/1 general rows lean_any >> $OUT/ab.log 2>&1 || { tail $OUT/ab.log; exit 1; }
CFG=c4 timeout -k 10 200 python3 tools/diag_shard_kernels.py 0/8 general rows lean >> $OUT/ab.log 2>&1 || { tail $OUT/ab.log; exit 1; }
grep -E "==|ms/pass" $OUT/ab.log
