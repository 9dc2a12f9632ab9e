bash scripts/gpu_iter.sh && bash scripts/gpu_pmc.sh bf16 4096 gpurun_out/pmc_bf16
