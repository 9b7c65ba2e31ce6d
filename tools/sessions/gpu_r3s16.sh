# 16-B lean stores: parity on the variant, then a same-box C4/C5 A/B at D=1
export TMPDIR=/tmp
OUT=gpurun_out/s16; mkdir -p $OUT
RCP_LIB_PATH=build_var/s16/librecoup_amd.so timeout -k 10 400 python3 -u -m pytest tests/test_gpu_lean.py tests/test_gpu_configs.py tests/test_gpu_rows.py -m gpu -x -q --timeout 120 --timeout-method thread --deselect tests/test_gpu_lean.py::test_lean_kernel_choice > $OUT/tests.log 2>&1; st=$?; tail -3 $OUT/tests.log; [ $st -eq 0 ] || exit $st
BENCH_ARGS="--inflight 1" bash tools/gpu_ab.sh $OUT "c4 c5" base s16 base s16
