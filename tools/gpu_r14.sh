VARIANTS=23,26,27,28,29,30 bash tools/gpu_round.sh r14
