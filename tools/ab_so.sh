# Same-box A/B of two builds of the library (abso/librecoup_amd_before.so vs the tree's) on C3
# passes (tools/diag_shard_kernels.py), alternating, after the row-wave tests
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_c3.py tests/test_gpu_rows.py tests/test_gpu_configs.py tests/test_gpu_rshim.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_so.log 2>&1 || { tail -30 gpurun_out/t_so.log; exit 1; }
tail -1 gpurun_out/t_so.log
for k in 1 2 3; do
  RCP_LIB_PATH=abso/librecoup_amd_before.so CFG=c3 timeout -k 10 200 python3 tools/diag_shard_kernels.py 0/1 auto 2>&1 | grep ms/pass | sed "s/^/before: /" || exit 1
  CFG=c3 timeout -k 10 200 python3 tools/diag_shard_kernels.py 0/1 auto 2>&1 | grep ms/pass | sed "s/^/after:  /" || exit 1
done
