# Round 3, GPU call j: customer-walk launch shapes around 2 waves per long group.
set -eu
O=gpurun_out/r03j
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python3 tools/walk_ab.py 2>/dev/null | tee $O/walk_base.json
for k in wa wb wc wd we wf wg; do timeout -k 10 200 python3 tools/with_lib.py tools/ab/libfdx_$k.so tools/walk_ab.py 2>/dev/null | tee $O/walk_$k.json; done
echo r03j done
