# copy threads per direction A/B on the host paths (C4): readset from unsorted reads in R's form,
# and the default e2e lines
set -o pipefail
for t in 8 12 16; do
  RCP_H2D_THREADS=$t timeout -k 10 200 python3 tools/diag_unsorted.py 3 codes+wruns 2>&1 | grep "readset 2" | sed "s/^/h2d $t: /"
done
for t in 8 12; do
  RCP_H2D_THREADS=$t timeout -k 10 400 python3 bench.py --no-cpu --steps 5 --inflight 1 > gpurun_out/abt_$t.json 2>/dev/null || exit 1
  python3 -c "
import json; d=json.load(open('gpurun_out/abt_$t.json')); e=d['e2e']
print('h2d $t e2e', round(e['ms'],2), 'any', round(e['any_order']['ms'],2), 'pipelined', round(e['samples_pipelined']['ms'],2), 'rle', round(e['rle_path']['ms'],2))"
done
