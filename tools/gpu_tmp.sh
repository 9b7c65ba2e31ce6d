export TMPDIR=/tmp
OUT=gpurun_out/ab8; mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1; tail -2 $OUT/tests.log
timeout -k 10 200 python3 tools/diag_c3.py > $OUT/rows.log 2>&1 && grep -v amdgpu $OUT/rows.log | cut -c1-70
timeout -k 10 300 python3 bench.py --config c3 --no-e2e > $OUT/c3_bench.json 2> $OUT/c3_bench.err; tail -c 600 $OUT/c3_bench.json
