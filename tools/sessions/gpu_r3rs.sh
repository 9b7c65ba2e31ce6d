#!/bin/bash
# readset_create phase times (timing build) in the C5 / C4 e2e legs
OUT=gpurun_out/r3rs
mkdir -p $OUT
export TMPDIR=/tmp
for c in c5 c4; do
RCP_LIB_PATH=build_var/tim/librecoup_amd.so timeout -k 10 600 python3 bench.py --config $c --no-cpu --steps 3 --warmup 1 --inflight 1 > $OUT/$c.json 2> $OUT/$c.err || { tail $OUT/$c.err; exit 1; }
done
grep -A12 "reads H2D" $OUT/c5.err | head -60
