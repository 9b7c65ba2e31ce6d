# GPU session of round 5: the full GPU suite (with the full-size C3 / C5 tests), the C4 bench
# line (e2e phases), C2 bench + SQ counters
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r5b}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=15 > $OUT/tests.log 2>&1 || { tail -80 $OUT/tests.log; exit 1; }
tail -25 $OUT/tests.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $OUT/c4_bench.json 2> $OUT/c4_bench.err && python -c "
import json; d=json.load(open('$OUT/c4_bench.json')); e=d['e2e']
print('C4', d['value'], d['ms_per_step'], d['config']['single_pass_ms'], d['roofline']['frac'])
print('e2e', round(e['ms'],2), e['equal_two_calls'], 'two calls', round(e['two_calls']['ms'],2), e['two_calls']['phases_ms'], 'pipelined', round(e['samples_pipelined']['ms'],2), e['samples_pipelined']['equal_one_shot'])
print('rle', round(e['rle_path']['ms'],2), e['rle_path']['phases_ms'], e['rle_path']['equal_fused'])"
timeout -k 10 300 python bench.py --config c2 --steps 50 --warmup 10 --no-e2e > $OUT/c2_bench.json 2> $OUT/c2_bench.err && python -c "import json; d=json.load(open('$OUT/c2_bench.json')); print('C2', d['value'], d['ms_per_step'], d['config']['single_pass_ms'], d['roofline']['frac'], d.get('kernel_ms'))"
PASSES=sq timeout -k 10 200 bash tools/pmc.sh $OUT/pmc c2 && python3 tools/pmc_sum.py $OUT/pmc 2>&1 | head -30
