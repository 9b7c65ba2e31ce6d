# Unsorted readset in R's form (codes + width runs) and with ends: codes and strands on the second
# H2D lane beside the starts (default) vs one lane (RCP_ONE_H2D_LANE=1); parity on the packed-upload tests
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_abi.py -m gpu -x -q -k "packed or readset" --timeout 200 --timeout-method thread > gpurun_out/t_h2d.log 2>&1 || { tail -30 gpurun_out/t_h2d.log; exit 1; }
tail -1 gpurun_out/t_h2d.log
for k in 1 2; do
  for v in two one; do
    if [ $v = one ]; then export RCP_ONE_H2D_LANE=1; else unset RCP_ONE_H2D_LANE; fi
    timeout -k 10 300 python3 tools/diag_unsorted.py 3 codes+wruns codes+ends > gpurun_out/un_$v.log 2>&1 || { tail gpurun_out/un_$v.log; exit 1; }
    grep -E "readset [12]:|h2d-packed|reads H2D" gpurun_out/un_$v.log | sed "s/^/$v: /"
  done
done
