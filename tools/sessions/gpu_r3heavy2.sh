bash tools/rocprof_ab.sh gpurun_out/heavy2 "c4" base t2k s2k s8k t2s2 base t2k s2k s8k t2s2
