# (record of a round-6 A/B: the RCP_NO_TILE_PERM knob was removed after it)
# C3 tile order: tiles holding interpolated genes first (default) vs natural order
# (RCP_NO_TILE_PERM=1): ms per pass alternating, then PMC traffic of both
set -o pipefail
for k in 1 2 3; do
  CFG=c3 timeout -k 10 200 python3 tools/diag_shard_kernels.py 0/1 auto 2>&1 | grep ms/pass | sed "s/^/perm:    /" || exit 1
  RCP_NO_TILE_PERM=1 CFG=c3 timeout -k 10 200 python3 tools/diag_shard_kernels.py 0/1 auto 2>&1 | grep ms/pass | sed "s/^/natural: /" || exit 1
done
for v in perm natural; do
  if [ $v = natural ]; then export RCP_NO_TILE_PERM=1; else unset RCP_NO_TILE_PERM; fi
  PASSES=traffic bash tools/pmc.sh gpurun_out/tp_$v c3 || exit 1
  python3 tools/pmc_traffic.py gpurun_out/tp_$v gpurun_out/tp_$v.json profiles/fetch_calib.json > /dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/tp_$v.json')); print('$v traffic', round(d['fetch_bytes']/1e6,1), round(d['write_bytes']/1e6,1), round(d['hbm_bytes_per_launch']/1e6,1))"
done
