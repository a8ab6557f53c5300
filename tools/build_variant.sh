#!/bin/bash
# Build an experiment variant of the product library with extra -D flags:
#   tools/build_variant.sh NAME -DFOO=1 ...   ->  tools/build/lib_NAME.so
# (objects in tools/build/obj_NAME; the in-tree product library is not touched)
set -e
name=$1; shift
root=$(cd "$(dirname "$0")/.." && pwd)
obj=$root/tools/build/obj_$name
mkdir -p "$obj"
cd "$root/aipstack_amd/csrc"
flags="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-parameter -I../../include -I. $*"
for f in chksum_kernels.hip frame_kernels.hip synth.hip chksum_host.cpp chksum_engine.cpp \
         chksum_engine_group.cpp host_threads.cpp; do
  /opt/rocm/bin/hipcc $flags -c $f -o "$obj/$f.o" &
done
g++ -std=c++17 -O3 -fPIC -c host_hook.cc -o "$obj/host_hook.cc.o" &
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -Wl,-rpath,/opt/rocm/lib -pthread -o "$root/tools/build/lib_$name.so" "$obj"/*.o
echo "built tools/build/lib_$name.so"
