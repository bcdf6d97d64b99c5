# Build an A/B variant of libfdx.so with extra compile-time defines (every source recompiled):
#   bash tools/build_ab.sh NAME "-DFDX_WALK_LP=2 -DFDX_EMIT_NT=0"  ->  tools/ab/libfdx_NAME.so
set -eu
NAME=$1; DEFS=$2
C=real-time_fraud_detection_system_amd/csrc
B=/tmp/fdx_ab/$NAME
mkdir -p tools/ab $B
rm -f $B/*.o
pids=""
for f in $C/*.hip $C/*.cpp; do
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -Iinclude $DEFS -c $f -o $B/$(basename $f).o &
    pids="$pids $!"
done
for p in $pids; do wait $p; done  # (set -e: a failed compile ends the script)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/ab/libfdx_$NAME.so $B/*.o
echo built tools/ab/libfdx_$NAME.so
