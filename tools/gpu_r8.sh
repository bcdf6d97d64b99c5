set -u
VARIANTS=1,5,6,7,8,9 bash tools/gpu_round.sh r8 || exit 1
bash tools/ring_sweep.sh
