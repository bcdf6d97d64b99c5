set -eu
O=gpurun_out/r03t
mkdir -p $O
timeout -k 10 300 python3 tools/host_profile.py 2>&1 | tee $O/host_profile.txt | tail -30
