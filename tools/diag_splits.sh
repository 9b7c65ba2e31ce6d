# C4 shards of the N = 1, 2, 4 splits: binned lean items of four 16-row rounds (default) vs two
# (RCP_LEAN_ROUNDS=2), ms per pass at D = 1, alternating, then bench steps with samples in flight
set -o pipefail
for k in 1 2; do
for s in ${SPECS:-0/4 0/2 0/1}; do
  timeout -k 10 300 python3 tools/diag_shard_kernels.py $s auto 2>&1 | grep ms/pass | sed 's/^/rounds4 /' || exit 1
  RCP_LEAN_ROUNDS=2 timeout -k 10 300 python3 tools/diag_shard_kernels.py $s auto 2>&1 | grep ms/pass | sed 's/^/rounds2 /' || exit 1
done
done
