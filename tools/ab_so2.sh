# Same-box A/B of two library builds (abso/librecoup_amd_before.so vs the tree's) on C2 and the
# C4 1/8 shard (tools/diag_shard_kernels.py), alternating, after the bin-difference tests
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_bins.py tests/test_gpu_random.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_so2.log 2>&1 || { tail -30 gpurun_out/t_so2.log; exit 1; }
tail -1 gpurun_out/t_so2.log
for k in 1 2 3; do
  for c in c2 c4; do
    s=0/1; [ $c = c4 ] && s=0/8
    RCP_LIB_PATH=abso/librecoup_amd_before.so CFG=$c timeout -k 10 200 python3 tools/diag_shard_kernels.py $s auto 2>&1 | grep ms/pass | sed "s/^/before: /" || exit 1
    CFG=$c timeout -k 10 200 python3 tools/diag_shard_kernels.py $s auto 2>&1 | grep ms/pass | sed "s/^/after:  /" || exit 1
  done
done
