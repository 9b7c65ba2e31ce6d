# PMC traffic of the C2 and C3 pileup kernels on the current tree (FETCH_SIZE, WRITE_SIZE passes)
set -o pipefail
for c in c2 c3; do
  PASSES=traffic bash tools/pmc.sh gpurun_out/traffic_$c $c || exit 1
  python3 tools/pmc_traffic.py gpurun_out/traffic_$c gpurun_out/traffic_$c.json profiles/fetch_calib.json || exit 1
done
