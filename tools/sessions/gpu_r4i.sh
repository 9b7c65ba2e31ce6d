#!/bin/bash
# round 4: locate ablations (timing only, wrong results): 1 no side writes, 2 no bucket searches,
# 4 no crange / record writes, 8 nothing after the row_info load; C2, C4 1/8, C4, C5 1/8
OUT=gpurun_out/r4i
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $OUT/tests.log 2>&1 || { tail -60 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for v in new nopre l1 l2 l4 l8; do
  lib=build_var/$v/librecoup_amd.so
  [ $v = new ] && lib=recoup_amd/librecoup_amd.so
  echo "== $v" >> $OUT/ab.log
  for spec in "c2 0/1" "c4 0/8" "c4 0/1" "c5 0/8"; do
    set -- $spec
    RCP_LIB_PATH=$lib CFG=$1 timeout -k 10 200 python3 tools/diag_shard_kernels.py $2 auto >> $OUT/ab.log 2>&1 || { tail $OUT/ab.log; exit 1; }
  done
done
for v in ring3 ring3b8; do
  RCP_LIB_PATH=build_var/$v/librecoup_amd.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_lean.py > $OUT/lean_$v.log 2>&1 || { tail -30 $OUT/lean_$v.log; exit 1; }
  tail -1 $OUT/lean_$v.log
  echo "== $v" >> $OUT/ab.log
  for spec in "c5 0/8" "c5 0/1" "c4 0/1"; do
    set -- $spec
    RCP_LIB_PATH=build_var/$v/librecoup_amd.so CFG=$1 timeout -k 10 200 python3 tools/diag_shard_kernels.py $2 auto >> $OUT/ab.log 2>&1 || { tail $OUT/ab.log; exit 1; }
  done
done
for v in bd8 bd16; do
  RCP_LIB_PATH=build_var/$v/librecoup_amd.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_bins.py > $OUT/bins_$v.log 2>&1 || { tail -30 $OUT/bins_$v.log; exit 1; }
  tail -1 $OUT/bins_$v.log
  echo "== $v" >> $OUT/ab.log
  RCP_LIB_PATH=build_var/$v/librecoup_amd.so CFG=c2 timeout -k 10 200 python3 tools/diag_shard_kernels.py 0/1 auto >> $OUT/ab.log 2>&1 || { tail $OUT/ab.log; exit 1; }
done
echo "== new" >> $OUT/ab.log
CFG=c2 timeout -k 10 200 python3 tools/diag_shard_kernels.py 0/1 auto >> $OUT/ab.log 2>&1 || { tail $OUT/ab.log; exit 1; }
grep -E "==|ms/pass" $OUT/ab.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o p -- python3 tools/diag_shard_kernels.py 0/8 auto > $OUT/prof.log 2>&1 || { tail $OUT/prof.log; exit 1; }
python3 - <<'PY'
import csv
for r in csv.DictReader(open('gpurun_out/r4i/prof/p_kernel_stats.csv')):
    if 'rcp_' in r['Name']:
        print(r['Name'][:50], r['Calls'], round(float(r['AverageNs'])/1000, 2), 'us')
PY
