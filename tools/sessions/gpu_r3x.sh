#!/bin/bash
# locate kernel ablations on C4 (rocprof kernel durations): a1 no side writes, a2 no bucket
# searches, a7 neither + no crange / record writes, a8 only the row_info load
OUT=gpurun_out/r3x
mkdir -p $OUT
export TMPDIR=/tmp
for v in base a1 a2 a7 a8; do
RCP_LIB_PATH=build_var/$v/librecoup_amd.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$v -o p -- \
  python3 bench.py --no-cpu --no-e2e --steps 30 --inflight 1 > $OUT/$v.json 2> $OUT/$v.err || { tail $OUT/$v.err; exit 1; }
echo "== $v"; grep -E "locate|heavy|lean" $OUT/$v/p_kernel_stats.csv | cut -d, -f1,2,4
done
