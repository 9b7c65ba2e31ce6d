#!/bin/bash
# Build compile-time variants of librecoup_amd.so into build_var/<name>/ and time the C4
# pileup for each (tools/diag_pileup.py quick).
#   tools/variants.sh build "name=-DFOO -DBAR" "name2=..."   (here, hipcc cross-compiles)
#   tools/variants.sh run name name2 ...                        (on the GPU box)
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/build_var
mode=$1; shift
if [ "$mode" = build ]; then
    [ -n "$KEEP" ] || rm -rf "$OUT"; mkdir -p "$OUT"
    for spec in "$@"; do
        name=${spec%%=*}; defs=${spec#*=}
        mkdir -p "$OUT/$name"
        (
        objs=""
        for src in rcp_kernels.hip rcp_rle.hip rcp_host.cpp rcp_stage.cpp rcp_bam.cpp; do
            /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -fvisibility=hidden -Wno-unused-result $defs \
                -c "$ROOT/recoup_amd/csrc/$src" -o "$OUT/$name/$src.o" || exit 1
            objs="$objs $OUT/$name/$src.o"
        done
        /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "$OUT/$name/librecoup_amd.so" $objs -lz -pthread &&
        rm -f $objs
        ) &
    done
    wait
    ls "$OUT"/*/librecoup_amd.so
    exit 0
fi
for v in "$@"; do
    echo "== $v"
    RCP_LIB_PATH=$OUT/$v/librecoup_amd.so timeout -k 10 150 python3 "$ROOT/tools/diag_pileup.py" quick
done
