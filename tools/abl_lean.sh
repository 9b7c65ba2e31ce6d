# Lean-kernel tuning sweep (GPU box): C4 and C5 pileup times under plan knobs.
set -e
run() { env "$@" timeout -k 10 150 python3 tools/diag_lean.py both 2>&1 | grep -v amdgpu.ids; }
run RCP_LEAN=1
run RCP_HEAVY_THRESHOLD=2048
run RCP_HEAVY_THRESHOLD=16384
