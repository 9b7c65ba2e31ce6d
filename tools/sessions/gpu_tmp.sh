export TMPDIR=/tmp
OUT=gpurun_out/e2e2; mkdir -p $OUT
RCP_LIB_PATH=build_var/ptime/librecoup_amd.so timeout -k 10 300 python3 tools/diag_e2e.py c4 > $OUT/diag.log 2>&1; grep -v amdgpu $OUT/diag.log | grep -v "0.0[0-9][0-9] ms" | tail -30
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1; tail -2 $OUT/tests.log
