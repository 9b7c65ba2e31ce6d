bash tools/rocprof_ab.sh gpurun_out/heavy "c4 c5 c2" base g1k g512 t8k t0 base g1k g512 t8k t0
