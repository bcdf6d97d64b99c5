# Round 3, GPU call as: ids past 2^key_bits through the fused path (rejected, no fault).
set -eu
O=gpurun_out/r03as
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_configs.py::test_fused_path_rejects_ids_out_of_range tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
echo r03as done
