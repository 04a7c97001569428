UB_POLICIES=1 timeout -k 10 120 tools/_bin/ubench_pattern > gpurun_out/${1:-r05pol}_pol.txt 2>&1; cat gpurun_out/${1:-r05pol}_pol.txt
