# Callers' matrices faulted in on a helper thread during the uploads (default) vs not
# (RCP_NO_PREFAULT=1): one call into a fresh matrix, into a touched one, three samples, the Rle
# path (tools/diag_stream.py, every call checked against a reference matrix)
set -o pipefail
for k in 1 2; do
  for v in pre none; do
    if [ $v = none ]; then export RCP_NO_PREFAULT=1; else unset RCP_NO_PREFAULT; fi
    timeout -k 10 300 python3 tools/diag_stream.py 6 > gpurun_out/pf_$v.log 2>&1 || { tail -20 gpurun_out/pf_$v.log; exit 1; }
    grep -E "median|mismatches" gpurun_out/pf_$v.log | sed "s/^/$v: /"
  done
done
