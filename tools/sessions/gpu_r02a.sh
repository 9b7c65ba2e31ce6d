#!/bin/bash
# Round-2 first GPU session: tests, PMC calibration, PCIe paths, bench N=1, N=2 rehearsal.
OUT=gpurun_out/r02a
mkdir -p $OUT
export TMPDIR=/tmp
{ nproc; python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)))"; cat /sys/fs/cgroup/cpu.max 2>&1;
  echo "OMP_NUM_THREADS=$OMP_NUM_THREADS"; grep -m1 "model name" /proc/cpuinfo; } > $OUT/host.txt 2>&1
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo TESTS FAILED; tail -30 $OUT/gpu_tests.log; exit 1; }
tail -3 $OUT/gpu_tests.log
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/calib/fetch -o p -- tools/fetch_calib > $OUT/calib_fetch.log 2>&1 &&
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/calib/write -o p -- tools/fetch_calib > $OUT/calib_write.log 2>&1 &&
python3 tools/pmc_calib.py $OUT/calib $OUT/fetch_calib.json || exit 1
timeout -k 10 300 tools/pcie_bench 1600 16 > $OUT/pcie.log 2>&1 || exit 1
cat $OUT/pcie.log
timeout -k 10 600 python3 bench.py > $OUT/c4_bench.json 2> $OUT/c4_bench.err || { tail $OUT/c4_bench.err; exit 1; }
cat $OUT/c4_bench.json
RCP_SHARE_GPU=1 RCP_DIST_BACKEND=gloo timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 10 --no-cpu --no-e2e --verify-gather \
    > $OUT/c4_n2_rehearsal.json 2> $OUT/c4_n2_rehearsal.err || { tail $OUT/c4_n2_rehearsal.err; exit 1; }
cat $OUT/c4_n2_rehearsal.json
