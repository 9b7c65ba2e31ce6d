#!/bin/bash
# C3 ablations (timing only, wrong results): boundary-position atomics skipped (nobound), all adds skipped (noadd)
OUT=gpurun_out/r04d
mkdir -p $OUT
export TMPDIR=/tmp
bash tools/gpu_ab.sh $OUT c3 base nobound noadd base nobound noadd
