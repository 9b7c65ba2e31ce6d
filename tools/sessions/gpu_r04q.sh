#!/bin/bash
# readset builds with pool-backed temporaries: C5 repeated builds, then the GPU tests
OUT=gpurun_out/r04q
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python tools/diag_readset.py c5 8 > $OUT/readset_c5.log 2>&1 || { tail $OUT/readset_c5.log; exit 1; }
grep -v amdgpu.ids $OUT/readset_c5.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/t.log 2>&1 || { tail -30 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
