#!/bin/bash
# Bench default D = auto (distinct samples in flight, agreed over ranks): N = 1 C4, 1/8 and 1/4 shards, N = 2 rehearsal (gloo, one GPU)
OUT=gpurun_out/r3q
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python bench.py --no-cpu > $OUT/c4_bench.json 2> $OUT/c4_bench.err || { tail $OUT/c4_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/c4_bench.json')); print('c4', d['value'], d['ms_per_step'], d['config']['samples'], d['config']['inflight_note'][-60:], d['config']['single_pass_ms'])"
for k in 0/8 7/8 0/4; do
timeout -k 10 300 python bench.py --no-cpu --no-e2e --sim-shard $k > $OUT/shard.json 2> $OUT/shard.err || { tail $OUT/shard.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/shard.json')); print('$k', d['ms_per_step'], d['config']['samples'], d['config']['inflight_note'][-60:])"
done
RCP_SHARE_GPU=1 RCP_DIST_BACKEND=gloo timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --no-cpu --no-e2e --steps 10 > $OUT/n2.out 2> $OUT/n2.err || { tail $OUT/n2.err; exit 1; }
grep metric $OUT/n2.out | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('n2', d['value'], d['ms_per_step'], d['config']['samples'], d['config']['inflight_note'][-60:])"
