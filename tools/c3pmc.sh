set -o pipefail
PASSES=sq bash tools/pmc.sh gpurun_out/c3pmc/v0 c3 && RCP_RW_VARIANT=4 PASSES=sq bash tools/pmc.sh gpurun_out/c3pmc/v4 c3 && RCP_RW_VARIANT=8 PASSES=sq bash tools/pmc.sh gpurun_out/c3pmc/v8 c3
