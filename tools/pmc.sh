#!/bin/bash
# Counter passes for the pileup kernel (one rocprofv3 run per pass; --pmc never combined with tracing).
# usage: tools/pmc.sh OUTDIR [config]
set -e
OUT=${1:-gpurun_out/pmc}
CFG=${2:-c4}
mkdir -p "$OUT"
export TMPDIR=/tmp
export PROF_META="$OUT/meta.json"
run() {  # $1 = pass name, rest = counters
    local name=$1; shift
    timeout -k 10 240 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o p -- python3 tools/prof_c4.py "$CFG" > "$OUT/$name.log" 2>&1
}
if [ "${PASSES:-all}" = traffic ]; then
  run fetch FETCH_SIZE
  run write WRITE_SIZE
  exit 0
fi
if [ "${PASSES:-all}" = sq ]; then
  run sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY
  run sq2 SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE
  exit 0
fi
run sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY
run sq2 SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE
run fetch FETCH_SIZE
run write WRITE_SIZE
run tcc TCC_HIT_sum TCC_MISS_sum
