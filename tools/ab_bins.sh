# (record of a round-6 A/B: the 4-wave variant was removed after it; RCP_BD_WAVES=16 remains)
# C2 bin-difference kernel: waves per 16-row tile (RCP_BD_WAVES 16 / 8 / 4; 8 and 4: the rows of a
# wave located in one chain of searches); parity on the bin-difference tests, then ms per pass
set -o pipefail
for w in 8 4; do
  RCP_BD_WAVES=$w timeout -k 10 300 python -u -m pytest tests/test_gpu_bins.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_bd$w.log 2>&1 || { tail -30 gpurun_out/t_bd$w.log; exit 1; }
  tail -1 gpurun_out/t_bd$w.log
done
for k in 1 2 3; do
  for w in 16 8 4; do
    RCP_BD_WAVES=$w CFG=c2 timeout -k 10 200 python3 tools/diag_shard_kernels.py 0/1 auto 2>&1 | grep ms/pass | sed "s/^/w$w: /" || exit 1
  done
done
