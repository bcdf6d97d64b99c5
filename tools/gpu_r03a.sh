# Round 3, first GPU call: forest row-order probe, blocked radix scatter A/B (bit-equality and
# time), compact terminal records end to end.  usage: bash tools/gpu_r03a.sh
set -eu
O=gpurun_out/r03a
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/radix_ab.py --out /tmp/radix_a.pt > $O/radix_a.json 2> $O/radix_a.err
cat $O/radix_a.json
FDX_RADIX_BLOCKED=1 timeout -k 10 300 python3 tools/radix_ab.py --out /tmp/radix_b.pt > $O/radix_b.json 2> $O/radix_b.err
cat $O/radix_b.json
python3 tools/radix_ab.py --compare /tmp/radix_a.pt /tmp/radix_b.pt | tee $O/radix_compare.json
rm -f /tmp/radix_a.pt /tmp/radix_b.pt
timeout -k 10 300 python3 tools/forest_order_probe.py > $O/order.json 2> $O/order.err
cat $O/order.json
AB_RUNS="base:FDX_OVERLAP=1 compact:FDX_TERM_COMPACT=1 blocked:FDX_RADIX_BLOCKED=1 both:FDX_TERM_COMPACT=1,FDX_RADIX_BLOCKED=1 base2:FDX_OVERLAP=1" \
    bash tools/gpu_ab.sh r03a/v1

timeout -k 10 900 python3 -u -m pytest tests/test_gpu_config1.py tests/test_gpu_parity.py tests/test_gpu_payload.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
echo r03a done
