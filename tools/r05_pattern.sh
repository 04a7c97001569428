#!/bin/bash
# Round 5: read rate of the scan's access pattern vs a contiguous one, through LDS-DMA / direct nt / direct loads.
O=gpurun_out/${1:-r05pat}; mkdir -p $O
timeout -k 10 120 tools/_bin/ubench_pattern > $O/pattern.txt 2>&1 || { cat $O/pattern.txt; exit 1; }
cat $O/pattern.txt
