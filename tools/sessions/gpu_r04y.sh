#!/bin/bash
# N = 2 rehearsal of the distributed bench on one GPU (gloo, two ranks sharing the device), with
# the per-rank e2e (width runs, pool-backed readsets) and the gather checked bit-equal to N = 1
OUT=gpurun_out/r04y
mkdir -p $OUT
export TMPDIR=/tmp
RCP_SHARE_GPU=1 RCP_DIST_BACKEND=gloo timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 10 --no-cpu --verify-gather \
    > $OUT/c4_n2_rehearsal.json 2> $OUT/c4_n2_rehearsal.err || { tail $OUT/c4_n2_rehearsal.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/c4_n2_rehearsal.json')); print(d['n_gpus'], round(d['ms_per_step'],4), '%.3e' % d['value'], d['gather'], round(d['e2e']['ms'],1), d['e2e']['width_runs'])"
