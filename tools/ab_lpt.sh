# (record of a round-6 A/B: the variant it selects was measured, not adopted, and removed from the
# library -- results under profiles/r06/; the script runs only against that build)
# Heaviest-first item order for binned lean plans of few 64-row items (default) vs per-XCD order
# (RCP_NO_BINNED_LPT=1): lean / random tests, then the C4 1/4 shards at D = 1 (diag) and with
# samples in flight auto (bench.py --sim-shard)
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_lean.py tests/test_gpu_random.py tests/test_gpu_configs.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_lpt.log 2>&1 || { tail -30 gpurun_out/t_lpt.log; exit 1; }
tail -1 gpurun_out/t_lpt.log
for k in 1 2; do
  for v in lpt xcd; do
    if [ $v = xcd ]; then export RCP_NO_BINNED_LPT=1; else unset RCP_NO_BINNED_LPT; fi
    timeout -k 10 200 python3 tools/diag_shard_kernels.py 1/4 auto 2>&1 | grep ms/pass | sed "s/^/$v: /" || exit 1
    timeout -k 10 300 python3 bench.py --sim-shard 1/4 --no-e2e --no-cpu > gpurun_out/lpt.json 2> gpurun_out/lpt.err || { tail -20 gpurun_out/lpt.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/lpt.json')); c=d['config']; print('$v step', round(d['ms_per_step'],4), 'D', c['inflight'], c['inflight_note'][-70:])"
  done
done
