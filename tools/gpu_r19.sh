bash tools/gpu_pmc.sh r19
