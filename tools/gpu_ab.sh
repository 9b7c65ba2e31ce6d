#!/bin/bash
# Same-box A/B of library variants in build_var/<name>/: tools/gpu_ab.sh OUTDIR "cfgs" v1 v2 ...
#   (bench.py --no-cpu --no-e2e per config and variant; one line per run; extra bench arguments
#   in $BENCH_ARGS, a tag for the file names in $TAG)
OUT=$1; CFGS=$2; shift 2
mkdir -p $OUT
for c in $CFGS; do
  for v in "$@"; do
    RCP_LIB_PATH=build_var/$v/librecoup_amd.so timeout -k 10 200 python3 bench.py --config $c --no-cpu --no-e2e --steps 30 $BENCH_ARGS > $OUT/${v}_$c$TAG.json 2> $OUT/${v}_$c$TAG.err || { tail $OUT/${v}_$c$TAG.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/${v}_$c$TAG.json')); print('$v $c $TAG', round(d['ms_per_step'],4), {k: round(x,4) for k,x in d['kernel_ms'].items()})" | tee -a $OUT/ab.log
  done
done
