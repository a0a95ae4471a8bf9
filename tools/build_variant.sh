#!/bin/bash
# Build a variant of libmivq.so with extra compiler flags, for interleaved A/Bs against the
# in-tree library (tools/ab_lib.py, tools/ab_opq.py).  usage: tools/build_variant.sh NAME "-DFOO=1 ..."
# -> tools/build/NAME.so (objects in tools/build/NAME/obj; nothing in the library tree changes)
set -eu
cd "$(dirname "$0")/.."
name=$1; shift
extra="$*"
src=vector-quantization_amd/csrc
obj=tools/build/$name/obj
mkdir -p $obj
flags="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -ffp-contract=off -Wall -Wno-unused-function -fvisibility=hidden -fno-gpu-rdc -fno-slp-vectorize $extra"
pids=()
for f in runtime pq pq_encode_cs sq rabitq rabitq_search adc opq extrabitq ivf; do
    /opt/rocm/bin/hipcc $flags -I include -c $src/$f.hip -o $obj/$f.o &
    pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/build/$name.so $obj/*.o
echo "built tools/build/$name.so ($extra)"
