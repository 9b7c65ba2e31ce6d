#!/bin/bash
# C3 interpolation: back substitution by the tabulated reciprocal (rcpdiv; parity tests first) vs the
# hardware division (base); ablations (timing only, wrong results): no fmm chains, no read pileup
OUT=gpurun_out/r04f
mkdir -p $OUT
export TMPDIR=/tmp
RCP_LIB_PATH=build_var/rcpdiv/librecoup_amd.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/rcpdiv_tests.log 2>&1 || { tail -30 $OUT/rcpdiv_tests.log; exit 1; }
tail -1 $OUT/rcpdiv_tests.log
bash tools/gpu_ab.sh $OUT c3 base rcpdiv nochain nodepth base rcpdiv nochain nodepth
