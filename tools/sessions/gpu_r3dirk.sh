# inline-key directory: full GPU suite on the in-tree build (q2), then a same-box C4/C2 A/B
export TMPDIR=/tmp
OUT=gpurun_out/dirk; mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1; st=$?; tail -3 $OUT/tests.log; [ $st -eq 0 ] || exit $st
BENCH_ARGS="--inflight 1" bash tools/gpu_ab.sh $OUT "c4 c2" base q2 q2w5 q4 base q2 q2w5 q4
