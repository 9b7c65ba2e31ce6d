# C3 row-wave kernel: two claimed rows' searches in one chain (RCP_RW_PAIR=1) vs one row at a
# time; parity on the row-wave tests in pair mode, then ms per pass alternating
set -o pipefail
RCP_RW_PAIR=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_c3.py tests/test_gpu_rows.py tests/test_gpu_configs.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_rwp.log 2>&1 || { tail -30 gpurun_out/t_rwp.log; exit 1; }
tail -1 gpurun_out/t_rwp.log
for k in 1 2 3; do
  CFG=c3 timeout -k 10 200 python3 tools/diag_shard_kernels.py 0/1 auto 2>&1 | grep ms/pass | sed "s/^/single: /" || exit 1
  RCP_RW_PAIR=1 CFG=c3 timeout -k 10 200 python3 tools/diag_shard_kernels.py 0/1 auto 2>&1 | grep ms/pass | sed "s/^/pair:   /" || exit 1
done
