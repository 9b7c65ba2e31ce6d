# Every shard of the N = 2, 4, 8 splits of C4 on one GPU (bench.py --sim-shard k/N, samples in
# flight auto): the slowest shard of a split sets that N's step in the driver's scaling run
set -o pipefail
OUT=${1:-gpurun_out/sweep}
mkdir -p "$OUT"
for spec in ${SPECS:-0/2 1/2 0/4 1/4 2/4 3/4 0/8 1/8 2/8 3/8 4/8 5/8 6/8 7/8}; do
  for kern in ${KERNELS:-auto}; do
  f="$OUT/shard_${spec/\//of}_$kern.json"
  timeout -k 10 200 python3 bench.py --sim-shard $spec --kernel $kern --no-e2e --no-cpu > "$f" 2> "$f.err" || { tail -20 "$f.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$f')); c=d['config']; print('$spec $kern', c['rank0_shard']['regions'], c['rank0_shard']['reads'], 'step', round(d['ms_per_step'],4), 'D', c['inflight'], 'pass', round(c['single_pass_ms'],4), d['roofline']['kernel'])"
  done
done
