#!/bin/bash
# A/B of library variants (GPU box): C4 pileup (tools/diag_lean.py) and the C5 / C3 bench lines
# per variant in build_var/<name>/.   tools/ab_variants.sh OUTDIR name1 name2 ...
set -e
OUT=$1; shift
mkdir -p "$OUT"
for v in "$@"; do
    lib=build_var/$v/librecoup_amd.so
    echo "== $v" | tee -a "$OUT/ab.log"
    RCP_LIB_PATH=$lib timeout -k 10 150 python3 tools/diag_lean.py 2>&1 | grep -v amdgpu.ids | tee -a "$OUT/ab.log"
    for c in ${AB_CONFIGS:-c5}; do
        RCP_LIB_PATH=$lib timeout -k 10 200 python3 bench.py --config $c --no-cpu --no-e2e --steps 20 \
            > "$OUT/${v}_$c.json" 2> "$OUT/${v}_$c.err"
        python3 -c "import json,sys; d=json.load(open('$OUT/${v}_$c.json')); print('$v $c', round(d['ms_per_step'],4), {k: round(x,4) for k,x in d['kernel_ms'].items()})" | tee -a "$OUT/ab.log"
    done
done
