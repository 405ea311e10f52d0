#!/bin/bash
# Build libcrdt_hip_<name>.so with extra compile definitions for the engine (A/B experiments):
#   tools/build_variant.sh v1 -DCRDT_DOC_LOG2S=1
set -e
cd "$(dirname "$0")/../crdt-benches_amd"
name=$1; shift
make -s -j8 libcrdt_hip.so
mkdir -p build/var_$name
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -I../include -Icsrc --offload-arch=gfx950 -munsafe-fp-atomics "$@" \
    -c csrc/engine.hip -o build/var_$name/engine.o
objs=$(ls build/*.o | grep -v "/engine.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o libcrdt_hip_$name.so build/var_$name/engine.o $objs \
    -lz -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo built libcrdt_hip_$name.so
