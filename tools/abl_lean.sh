# Lean-kernel tuning sweep (GPU box): library variants x plan knobs, C4 pileup times.
set -e
run() { env "$@" timeout -k 10 150 python3 tools/diag_lean.py both 2>&1 | grep -v amdgpu.ids; }
run RCP_LEAN=1
run RCP_LIB_PATH=build_var/nosearch/librecoup_amd.so
run RCP_LIB_PATH=build_var/locwpe4/librecoup_amd.so
run RCP_HEAVY_THRESHOLD=0
