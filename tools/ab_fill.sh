# (record of a round-6 A/B: the variant it selects was measured, not adopted, and removed from the
# library -- results under profiles/r06/; the script runs only against that build)
# Concurrent plans' share of the workgroup slots (RCP_GRID_FILL eighths; 7 = default) on the C4
# full table and its 1/2 and 1/4 shards, samples in flight auto (bench.py --sim-shard)
set -o pipefail
for s in 0/4 0/2 0/1; do
  for f in 7 6 5; do
    RCP_GRID_FILL=$f timeout -k 10 300 python3 bench.py --sim-shard $s --no-e2e --no-cpu > gpurun_out/fill.json 2> gpurun_out/fill.err || { tail -20 gpurun_out/fill.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/fill.json')); c=d['config']; print('$s fill $f step', round(d['ms_per_step'],4), 'D', c['inflight'], c['inflight_note'][-60:])"
  done
done
