#!/bin/bash
# A/B of one library under environment variants (GPU box):
#   tools/ab_env.sh OUTDIR "configs" "NAME=ENV ..." ...
# e.g. tools/ab_env.sh gpurun_out/ab "c4 c2" "lpr1=RCP_LOC_LPR=1" "lpr4=RCP_LOC_LPR=4"
set -e
OUT=$1; shift
CONFIGS=$1; shift
mkdir -p "$OUT"
for spec in "$@"; do
    name=${spec%%=*}
    envs=${spec#*=}
    for c in $CONFIGS; do
        env $envs timeout -k 10 200 python3 bench.py --config $c --no-cpu --no-e2e --steps 20 \
            > "$OUT/${name}_$c.json" 2> "$OUT/${name}_$c.err"
        python3 -c "import json; d=json.load(open('$OUT/${name}_$c.json')); print('$name $c', round(d['ms_per_step'],4), {k: round(x,4) for k,x in d['kernel_ms'].items()})" | tee -a "$OUT/ab.log"
    done
done
