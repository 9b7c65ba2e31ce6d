#!/bin/bash
# e2e host path diagnostics + strong-scaling shard rehearsal + bench with rocprof
OUT=gpurun_out/r02b
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/diag_e2e.py c4 > $OUT/diag_e2e_c4.log 2>&1 || { tail $OUT/diag_e2e_c4.log; exit 1; }
cat $OUT/diag_e2e_c4.log | grep -v amdgpu.ids
for k in 0 3 7; do
  timeout -k 10 300 python3 bench.py --sim-shard $k/8 --no-cpu --no-e2e > $OUT/shard_${k}of8.json 2> $OUT/shard_${k}of8.err || { tail $OUT/shard_${k}of8.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/shard_${k}of8.json')); print('shard $k/8', d['config']['rank0_shard'], round(d['ms_per_step'],4), {k: round(v,4) for k,v in d['kernel_ms'].items()})"
done
timeout -k 10 300 python3 bench.py --sim-shard 0/2 --no-cpu --no-e2e > $OUT/shard_0of2.json 2>/dev/null && python3 -c "import json; d=json.load(open('$OUT/shard_0of2.json')); print('shard 0/2', round(d['ms_per_step'],4), d['kernel_ms'])"
timeout -k 10 300 python3 bench.py --sim-shard 0/4 --no-cpu --no-e2e > $OUT/shard_0of4.json 2>/dev/null && python3 -c "import json; d=json.load(open('$OUT/shard_0of4.json')); print('shard 0/4', round(d['ms_per_step'],4), d['kernel_ms'])"
