set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5a
timeout -k 10 400 python -u -m pytest tests/test_gpu_shards.py tests/test_gpu_rshim.py tests/test_gpu_bins.py tests/test_gpu_lean.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5a/tests.log 2>&1 || { tail -60 gpurun_out/r5a/tests.log; exit 1; }
tail -3 gpurun_out/r5a/tests.log
timeout -k 10 300 python bench.py --config c2 --steps 50 --warmup 10 > gpurun_out/r5a/c2_bench.json 2> gpurun_out/r5a/c2_bench.err && cat gpurun_out/r5a/c2_bench.json | python -c "import json,sys; d=json.load(sys.stdin); print(d['value'], d['ms_per_step'], d['config']['single_pass_ms'], d['roofline'], d.get('kernel_ms'))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5a/prof -o c2 -- python3 bench.py --config c2 --no-cpu --no-e2e --inflight 1 --steps 50 > gpurun_out/r5a/c2_prof.json 2> gpurun_out/r5a/c2_prof.err
find gpurun_out/r5a/prof -name "*kernel_stats.csv" | head -3 | xargs -I{} sh -c 'head -8 {}'
PASSES=sq timeout -k 10 200 bash tools/pmc.sh gpurun_out/r5a/pmc c2 && python3 tools/pmc_sum.py gpurun_out/r5a/pmc 2>&1 | head -30
