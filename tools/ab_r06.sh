set -o pipefail
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_uns2.log 2>&1; tail -3 gpurun_out/t_uns2.log
timeout -k 10 300 python3 tools/diag_unsorted.py 3 codes+ends codes+wruns > gpurun_out/unsorted2.log 2>&1; grep -E "readset [0-9]|h2d-packed|\[plan\] reads|\[plan\] merged" gpurun_out/unsorted2.log | tail -16
for r in 1 2 4; do RCP_GEN_ROUNDS=$r timeout -k 10 200 python3 tools/diag_shard_kernels.py 0/8 general 2>&1 | grep ms/pass | sed "s/^/rounds $r: /"; done
