# GPU parity under every MaskL-index mode, then warm A/B of the modes on C1 and C3
set -e
for m in 1 2 0; do
  CDC_MASKL_INDEX=$m timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_mode$m.txt 2>&1
  tail -1 gpurun_out/gpu_mode$m.txt
done
bash tools/ab_env_warm.sh CDC_MASKL_INDEX "0 1 2" > gpurun_out/ab_l3_c1.txt 2>&1
bash tools/ab_env_warm.sh CDC_MASKL_INDEX "0 1 2" --workload c3 > gpurun_out/ab_l3_c3.txt 2>&1
