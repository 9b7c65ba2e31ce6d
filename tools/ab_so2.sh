# Same-box A/B of two library builds (abso/librecoup_amd_before.so vs the tree's) on the C4 1/8
# and 1/4 shards (tools/diag_shard_kernels.py; general kernel with the locate folded in), after
# the random-table, shard and bin-difference tests
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_random.py tests/test_gpu_shards.py tests/test_gpu_bins.py tests/test_gpu_abi.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_so2.log 2>&1 || { tail -30 gpurun_out/t_so2.log; exit 1; }
tail -1 gpurun_out/t_so2.log
for k in 1 2 3; do
  RCP_LIB_PATH=abso/librecoup_amd_before.so timeout -k 10 200 python3 tools/diag_shard_kernels.py 0/8 auto 2>&1 | grep ms/pass | sed "s/^/before: /" || exit 1
  timeout -k 10 200 python3 tools/diag_shard_kernels.py 0/8 auto 2>&1 | grep ms/pass | sed "s/^/after:  /" || exit 1
done
