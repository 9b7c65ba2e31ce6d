# (record of a round-6 A/B: the variant it selects was measured, not adopted, and removed from the
# library -- results under profiles/r06/; the script runs only against that build)
# Binned lean fold plans with the skewed chunks deferred (default) vs the locate + heavy path
# (RCP_NO_LEAN_DEFER=1) vs the build before (abso/librecoup_amd_before.so): lean tests in both
# modes (RCP_DEFER_MIN=64: small tables defer), then C4 passes (full and 1/4, 1/8 shards)
set -o pipefail
RCP_DEFER_MIN=64 timeout -k 10 300 python -u -m pytest tests/test_gpu_lean.py tests/test_gpu_random.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_def.log 2>&1 || { tail -40 gpurun_out/t_def.log; exit 1; }
tail -1 gpurun_out/t_def.log
for k in 1 2; do
  for s in 0/1 0/4 0/8; do
    RCP_LIB_PATH=abso/librecoup_amd_before.so timeout -k 10 200 python3 tools/diag_shard_kernels.py $s auto lean 2>&1 | grep ms/pass | sed "s/^/before: /" || exit 1
    RCP_NO_LEAN_DEFER=1 timeout -k 10 200 python3 tools/diag_shard_kernels.py $s auto lean 2>&1 | grep ms/pass | sed "s/^/nodefer: /" || exit 1
    timeout -k 10 200 python3 tools/diag_shard_kernels.py $s auto lean 2>&1 | grep ms/pass | sed "s/^/defer:  /" || exit 1
  done
done
