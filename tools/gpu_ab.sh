#!/bin/bash
# A/B of library variants on C3 (tools/diag_c3.py) + optional bench configs, then the GPU tests
# of the default build.   tools/gpu_ab.sh OUTDIR "c3 c4" name1 name2 ...
OUT=$1; shift
CFGS=$1; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in "$@"; do
    lib=build_var/$v/librecoup_amd.so
    for c in $CFGS; do
        if [ "$c" = c3diag ]; then
            RCP_LIB_PATH=$lib timeout -k 10 200 python3 tools/diag_c3.py > "$OUT/${v}_c3diag.log" 2>&1 || { tail "$OUT/${v}_c3diag.log"; exit 1; }
            echo "== $v c3diag"; grep -v amdgpu.ids "$OUT/${v}_c3diag.log"
            continue
        fi
        RCP_LIB_PATH=$lib timeout -k 10 200 python3 bench.py --config $c --no-cpu --no-e2e --steps 20 \
            > "$OUT/${v}_$c.json" 2> "$OUT/${v}_$c.err" || { tail "$OUT/${v}_$c.err"; exit 1; }
        python3 -c "import json,sys; d=json.load(open('$OUT/${v}_$c.json')); print('$v $c', round(d['ms_per_step'],4), {k: round(x,4) for k,x in d['kernel_ms'].items()}, 'parity', d.get('parity_sample'))"
    done
done
if [ -n "$GPU_TESTS" ]; then
    timeout -k 10 600 python3 -u -m pytest $GPU_TESTS -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
    tail -2 $OUT/gpu_tests.log
fi
