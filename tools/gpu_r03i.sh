# Round 3, GPU call i: customer-walk launch shapes (tools/ab builds), bit-identical digests.
set -eu
O=gpurun_out/r03i
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python3 tools/walk_ab.py > $O/walk_base.json 2>&1; cat $O/walk_base.json
for k in 1 2 3 4; do timeout -k 10 200 python3 tools/with_lib.py tools/ab/libfdx_walk$k.so tools/walk_ab.py > $O/walk_$k.json 2>&1; cat $O/walk_$k.json; done
echo r03i done
