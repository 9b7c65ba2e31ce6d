#!/bin/bash
# round 4: the R-shim / API GPU tests (dimnames), then the baseline shard rehearsals (gpu_r4a.sh)
OUT=gpurun_out/r4b
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_rshim.py tests/test_gpu_api.py > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
bash tools/sessions/gpu_r4a.sh
