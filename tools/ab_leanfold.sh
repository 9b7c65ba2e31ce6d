# C5 / C4 1/8 shards: per-base lean plans with the searches folded into the claim vs the locate launch
set -o pipefail
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_lf.log 2>&1; tail -3 gpurun_out/t_lf.log
for k in 1 2; do
  CFG=c5 timeout -k 10 200 python3 tools/diag_shard_kernels.py 0/8 auto 2>&1 | grep ms/pass | sed "s/^/fold: /"
  RCP_NO_LEAN_FOLD=1 CFG=c5 timeout -k 10 200 python3 tools/diag_shard_kernels.py 0/8 auto 2>&1 | grep ms/pass | sed "s/^/locate: /"
done
timeout -k 10 200 python3 tools/diag_shard_kernels.py 0/8 auto 2>&1 | grep ms/pass
