bash tools/gpu_round.sh r29 && bash tools/gpu_pmc.sh r29
