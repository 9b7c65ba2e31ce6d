#!/bin/bash
# A/B: general pileup kernel rounds per workgroup (base = auto 2/1, r1, r4) on C2 and the 1/8, 1/4 C4 shards
OUT=gpurun_out/r3f2
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
for v in base r1 r4; do
  lib=build_var/$v/librecoup_amd.so
  for c in c2 s8; do
    if [ $c = c2 ]; then a="--config c2"; else a="--sim-shard 0/8"; fi
    for d in 1 auto; do
      RCP_LIB_PATH=$lib timeout -k 10 200 python3 bench.py $a --no-cpu --no-e2e --inflight $d --steps 20 > $OUT/${v}_${c}_$d.json 2> $OUT/${v}_${c}_$d.err || { tail $OUT/${v}_${c}_$d.err; exit 1; }
      python3 -c "import json; d=json.load(open('$OUT/${v}_${c}_$d.json')); print('$v $c D=$d', round(d['ms_per_step'],4), 'single', round(d['config']['single_pass_ms'],4), {k: round(x,4) for k,x in d['kernel_ms'].items()}, 'parity', d.get('parity_sample'))" | tee -a $OUT/ab.log
    done
  done
done
done
