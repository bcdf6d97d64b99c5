VARIANTS=23,24,25,16 bash tools/gpu_round.sh r13 && bash tools/gpu_pmc.sh r13
