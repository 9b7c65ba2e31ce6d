# (record of a round-6 ablation: abso/lib_abl.so was a build without the stage stores)
set -o pipefail
for k in 1 2 3; do
  RCP_LIB_PATH=abso/lib_base.so CFG=c3 timeout -k 10 200 python3 tools/diag_shard_kernels.py 0/1 auto 2>&1 | grep ms/pass | sed "s/^/base: /" || exit 1
  RCP_LIB_PATH=abso/lib_abl.so CFG=c3 timeout -k 10 200 python3 tools/diag_shard_kernels.py 0/1 auto 2>&1 | grep ms/pass | sed "s/^/nostage: /" || exit 1
done
