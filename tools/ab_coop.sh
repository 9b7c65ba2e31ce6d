# C4 1/8 shard, general kernel with the locate folded in: the cooperative-row threshold
# (RCP_COOP_MIN candidates a chunk; 8192 default), ms per pass at D = 1
set -o pipefail
for k in 1 2; do
  for c in 2048 4096 8192 16384 65536; do
    RCP_COOP_MIN=$c timeout -k 10 200 python3 tools/diag_shard_kernels.py 0/8 auto 2>&1 | grep ms/pass | sed "s/^/coop $c: /" || exit 1
  done
done
