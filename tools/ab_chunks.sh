# (record of a round-6 A/B: the variant it selects was measured, not adopted, and removed from the
# library -- results under profiles/r06/; the script runs only against that build)
# C5 1/8 shard (per-base lean plan with the searches folded into the claim): column chunks
# capped at 16 (the crange table's limit, RCP_FOLD_MAX_CHUNKS=16) vs 64; parity on the lean tests
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_lean.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_ch.log 2>&1 || { tail -30 gpurun_out/t_ch.log; exit 1; }
tail -1 gpurun_out/t_ch.log
for k in 1 2 3; do
  RCP_FOLD_MAX_CHUNKS=16 CFG=c5 timeout -k 10 200 python3 tools/diag_shard_kernels.py 0/8 auto 2>&1 | grep ms/pass | sed "s/^/max16: /" || exit 1
  CFG=c5 timeout -k 10 200 python3 tools/diag_shard_kernels.py 0/8 auto 2>&1 | grep ms/pass | sed "s/^/max64: /" || exit 1
done
CFG=c5 timeout -k 10 200 python3 tools/diag_shard_kernels.py 0/1 auto 2>&1 | grep ms/pass | sed "s/^/full: /" || exit 1
