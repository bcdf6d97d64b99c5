# Build A/B variants of libfdx.so that differ in one compile-time define of fdx_windows.hip:
#   bash tools/build_ab.sh NAME "-DFDX_WALK_SHAPE=2"   ->  tools/ab/libfdx_NAME.so
# (the other objects are the in-tree build's; run `make -C real-time_fraud_detection_system_amd/csrc` first)
set -eu
NAME=$1; DEFS=$2
C=real-time_fraud_detection_system_amd/csrc
mkdir -p tools/ab /tmp/fdx_ab
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -Iinclude $DEFS -c $C/fdx_windows.hip -o /tmp/fdx_ab/windows_$NAME.o
objs=$(ls $C/build/*.o | grep -v fdx_windows)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/ab/libfdx_$NAME.so $objs /tmp/fdx_ab/windows_$NAME.o
echo built tools/ab/libfdx_$NAME.so
