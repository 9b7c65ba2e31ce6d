# Per-base lean fold vs the locate launch (RCP_NO_LEAN_FOLD=1) on the full C5 table (25 k rows:
# plans in flight keep the locate now) and its 1/8 shard (3 k rows: folded in both uses), bench
# steps with samples in flight auto
set -o pipefail
for k in 1 2; do
  for s in 0/1 0/8; do
    for v in default locate; do
      if [ $v = locate ]; then export RCP_NO_LEAN_FOLD=1; else unset RCP_NO_LEAN_FOLD; fi
      timeout -k 10 300 python3 bench.py --config c5 --sim-shard $s --no-e2e --no-cpu > gpurun_out/c5f.json 2> gpurun_out/c5f.err || { tail -20 gpurun_out/c5f.err; exit 1; }
      python3 -c "import json; d=json.load(open('gpurun_out/c5f.json')); c=d['config']; print('$s $v step', round(d['ms_per_step'],4), 'D', c['inflight'], 'pass', round(c['single_pass_ms'],4), c['inflight_note'][-70:])"
    done
  done
done
