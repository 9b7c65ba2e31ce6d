#!/bin/bash
# round 4: GPU tests; A/B of new (heaviest-first lean items, lockstep rounds of 8 for > 8 chunks) vs nolpt / ks4 on the shards
OUT=gpurun_out/r4h
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $OUT/tests.log 2>&1 || { tail -60 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for v in new nolpt ks4 new nolpt; do
  lib=build_var/$v/librecoup_amd.so
  [ $v = new ] && lib=recoup_amd/librecoup_amd.so
  echo "== $v" >> $OUT/ab.log
  for spec in "c5 0/8" "c5 7/8" "c4 0/8" "c2 0/1"; do
    set -- $spec
    RCP_LIB_PATH=$lib CFG=$1 timeout -k 10 200 python3 tools/diag_shard_kernels.py $2 auto >> $OUT/ab.log 2>&1 || { tail $OUT/ab.log; exit 1; }
  done
done
grep -E "==|ms/pass" $OUT/ab.log
timeout -k 10 300 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'],d['ms_per_step'],d['config']['single_pass_ms'],d['kernel_ms'],d['inflight_check'],d['parity_sample']['ok'])"
# SQ counters of the C5 1/8 shard's kernels
export SHARD=0/8
PASSES=sq bash tools/pmc.sh $OUT/pmc_c5s c5 || { tail $OUT/pmc_c5s/*.log; exit 1; }
python3 tools/pmc_sum.py -k rcp_ $OUT/pmc_c5s > $OUT/pmc_c5s.txt
cat $OUT/pmc_c5s.txt
