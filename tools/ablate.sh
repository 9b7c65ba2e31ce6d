#!/bin/bash
# Build ablation variants of librecoup_amd.so (one phase of the pileup kernel removed each)
# into build_abl/<name>/ and time the C4 pileup for each.  Diagnostic only: the outputs of
# an ablated build are wrong by construction.
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/build_abl
mkdir -p "$OUT"
build() {  # name, defines...
    local name=$1; shift
    mkdir -p "$OUT/$name"
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -fvisibility=hidden -Wno-unused-result "$@" \
        -c "$ROOT/recoup_amd/csrc/rcp_kernels.hip" -o "$OUT/$name/k.o"
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -fvisibility=hidden -Wno-unused-result \
        -c "$ROOT/recoup_amd/csrc/rcp_host.cpp" -o "$OUT/$name/h.o"
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "$OUT/$name/librecoup_amd.so" "$OUT/$name/k.o" "$OUT/$name/h.o"
}
if [ "$1" = "build" ]; then
    build base &
    build no_atomics -DRCP_ABL_ATOMICS &
    build no_scan -DRCP_ABL_SCAN &
    build no_bins -DRCP_ABL_BINS &
    build no_epi -DRCP_ABL_EPI &
    build no_all -DRCP_ABL_ATOMICS -DRCP_ABL_SCAN -DRCP_ABL_BINS -DRCP_ABL_EPI &
    wait
    exit 0
fi
for v in base no_atomics no_scan no_bins no_epi no_all; do
    echo "== $v"
    RCP_LIB_PATH=$OUT/$v/librecoup_amd.so timeout -k 10 120 python3 "$ROOT/tools/diag_pileup.py" quick
done
