#!/bin/bash
# Pipelined two-block execution (locate of block 1 under block 0's pileup): GPU tests, A/B vs RCP_PIPE=0, block share sweep, 1/8 shard
OUT=gpurun_out/r3i
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
run() {  # tag, env..., bench args
  local tag=$1; shift
  env "$@" > /dev/null
  timeout -k 10 200 env $ENVS python3 bench.py --no-cpu --no-e2e --steps 30 $ARGS > $OUT/$tag.json 2> $OUT/$tag.err || { tail $OUT/$tag.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$tag.json')); print('$tag', round(d['ms_per_step'],4), d['parity_sample'], {k: round(x,4) for k,x in d['kernel_ms'].items()})" | tee -a $OUT/ab.log
}
for rep in 1 2; do
  for c in c4 c5; do
    ENVS="RCP_PIPE=0" ARGS="--config $c" run ${c}_nopipe_$rep
    ENVS="RCP_PIPE=1" ARGS="--config $c" run ${c}_pipe25_$rep
    ENVS="RCP_PIPE_FRAC=0.125" ARGS="--config $c" run ${c}_pipe12_$rep
    ENVS="RCP_PIPE_FRAC=0.4" ARGS="--config $c" run ${c}_pipe40_$rep
  done
  ENVS="RCP_PIPE=0" ARGS="--sim-shard 0/8" run shard8_nopipe_$rep
  ENVS="RCP_PIPE=1" ARGS="--sim-shard 0/8" run shard8_pipe25_$rep
  ENVS="RCP_PIPE_FRAC=0.4" ARGS="--sim-shard 0/8" run shard8_pipe40_$rep
done
