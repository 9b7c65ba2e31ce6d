# (record of a round-6 A/B: the variant it selects was measured, not adopted, and removed from the
# library -- results under profiles/r06/; the script runs only against that build)
# C3 row-wave kernel: run-merged adds over consecutive candidates (RCP_RW_RUNS=1) vs interleaved
# slots with one atomic per read; parity on the row-wave tests in runs mode, ms per pass alternating,
# and the SQ counters of both
set -o pipefail
RCP_RW_RUNS=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_c3.py tests/test_gpu_rows.py tests/test_gpu_configs.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_rwr.log 2>&1 || { tail -30 gpurun_out/t_rwr.log; exit 1; }
tail -1 gpurun_out/t_rwr.log
for k in 1 2 3; do
  CFG=c3 timeout -k 10 200 python3 tools/diag_shard_kernels.py 0/1 auto 2>&1 | grep ms/pass | sed "s/^/atomics: /" || exit 1
  RCP_RW_RUNS=1 CFG=c3 timeout -k 10 200 python3 tools/diag_shard_kernels.py 0/1 auto 2>&1 | grep ms/pass | sed "s/^/runs:    /" || exit 1
done
RCP_RW_RUNS=1 PASSES=sq bash tools/pmc.sh gpurun_out/c3pmc/runs c3
