# C4 / C5 1/8 shards (D = 1) on several pileup kernels, and rocprofv3 kernel summaries of them
set -o pipefail
O=${1:-gpurun_out/shp}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/diag_shard_kernels.py 0/8 general general:0:4096 lean > $O/c4.log 2>&1 || { tail -20 $O/c4.log; exit 1; }
grep ms/pass $O/c4.log
CFG=c5 timeout -k 10 300 python3 tools/diag_shard_kernels.py 0/8 auto general general:0:4096 > $O/c5.log 2>&1 || { tail -20 $O/c5.log; exit 1; }
grep ms/pass $O/c5.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof4 -o p -- python3 tools/diag_shard_kernels.py 0/8 general general:0:4096 > $O/c4p.log 2>&1 || exit 1
grep -h "rcp_pileup\|rcp_locate\|rcp_heavy" $O/prof4/p_kernel_stats.csv | cut -d, -f1-4
