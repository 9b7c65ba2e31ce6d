# C3 row-wave ablations: RCP_RW_V6 no splines, RCP_RW_V7 spline results stored contiguously (wrong cells)
set -o pipefail
for k in 1 2 3; do
  CFG=c3 timeout -k 10 200 python3 tools/diag_shard_kernels.py 0/1 auto 2>&1 | grep ms/pass | sed "s/^/v0: /" || exit 1
  RCP_RW_V6=1 CFG=c3 timeout -k 10 200 python3 tools/diag_shard_kernels.py 0/1 auto 2>&1 | grep ms/pass | sed "s/^/v6: /" || exit 1
  RCP_RW_V7=1 CFG=c3 timeout -k 10 200 python3 tools/diag_shard_kernels.py 0/1 auto 2>&1 | grep ms/pass | sed "s/^/v7: /" || exit 1
done
