#!/bin/bash
# C2 general kernel skeleton (-DRCP_GEN_ABL=3: no read loads / adds, no output stores; wrong
# results, timing and counters only): its instruction mix against the full kernel's (r3f7)
OUT=gpurun_out/r3f8
mkdir -p $OUT
export TMPDIR=/tmp
RCP_LIB_PATH=build_var/none/librecoup_amd.so timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY --output-format csv -d $OUT/pmc/sq1 -o p -- python3 tools/prof_c4.py c2 > $OUT/sq1.log 2>&1 || { tail $OUT/sq1.log; exit 1; }
python3 tools/pmc_kernels.py $OUT/pmc pileup > $OUT/c2_skeleton_sq.txt 2>&1
cat $OUT/c2_skeleton_sq.txt
