#!/bin/bash
# PMC calibration incl. 4-B int32 reads (uniform-width starts); then the directory A/B on shards
OUT=gpurun_out/r3cal
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o p -- tools/fetch_calib > $OUT/fetch.log 2>&1 || { tail $OUT/fetch.log; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o p -- tools/fetch_calib > $OUT/write.log 2>&1 || { tail $OUT/write.log; exit 1; }
python3 tools/pmc_calib.py $OUT $OUT/fetch_calib.json | head -12
bash tools/sessions/gpu_r3d2.sh
CFG=c2 timeout -k 10 300 python3 tools/diag_shard_kernels.py 0/1 auto rows lean_any > $OUT/c2_kernels.log 2> $OUT/c2_kernels.err || { tail $OUT/c2_kernels.err; exit 1; }
cat $OUT/c2_kernels.log
