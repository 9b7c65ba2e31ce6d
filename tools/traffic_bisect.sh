# C3 row-wave PMC traffic per library build (abso/lib_*.so: before the round-6 row-wave changes,
# after the epilogue change, after the flush change; the tree's own library last)
set -o pipefail
for v in base epi flush tree; do
  if [ $v = tree ]; then unset RCP_LIB_PATH; else export RCP_LIB_PATH=abso/lib_$v.so; fi
  PASSES=traffic bash tools/pmc.sh gpurun_out/tb_$v c3 || exit 1
  python3 tools/pmc_traffic.py gpurun_out/tb_$v gpurun_out/tb_$v.json profiles/fetch_calib.json > /dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/tb_$v.json')); print('$v', round(d['fetch_bytes']/1e6,1), round(d['write_bytes']/1e6,1), round(d['hbm_bytes_per_launch']/1e6,1))"
done
