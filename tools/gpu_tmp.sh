export TMPDIR=/tmp
OUT=gpurun_out/t10; mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1; tail -3 $OUT/tests.log
