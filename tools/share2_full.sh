# 2 ranks sharing the one GPU with the default flags (host-path e2e per rank on its shard, as the
# driver's scaling run would do on 2 GPUs)
set -o pipefail
RCP_SHARE_GPU=1 timeout -k 10 900 python3 bench.py --gpus 2 > gpurun_out/share2_full.json 2> gpurun_out/share2_full.err || { tail -30 gpurun_out/share2_full.err; exit 1; }
python3 -c "import json; d=json.loads([l for l in open('gpurun_out/share2_full.json') if l.startswith('{')][-1]); print(d['n_gpus'], d['value'], d['ms_per_step'], d['e2e']['ms'], d['e2e'].get('note','')[-60:])"
