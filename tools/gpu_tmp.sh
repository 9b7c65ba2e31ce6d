export TMPDIR=/tmp
OUT=gpurun_out/ab5; mkdir -p $OUT
timeout -k 10 200 python3 tools/diag_c3.py > $OUT/rows.log 2>&1 && grep -v amdgpu $OUT/rows.log &&
DIAG_KERNEL=general timeout -k 10 200 python3 tools/diag_c3.py all > $OUT/gen.log 2>&1 && grep -v amdgpu $OUT/gen.log &&
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_rows.py tests/test_gpu_c3.py tests/test_gpu_lean.py -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1; tail -3 $OUT/tests.log
