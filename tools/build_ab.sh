#!/bin/bash
# Builds an A/B variant of libmivq.so: tools/build_ab.sh NAME "-DFOO=1 ..." [source.hip]
# Compiles the given source (default pq_encode_cs.hip) with the extra flags, links it with the
# in-tree objects of the other sources into vector-quantization_amd/lib/ab/libmivq_NAME.so
# (travels to the GPU box with the tree; git-ignored like every .so).
set -eu
cd "$(dirname "$0")/../vector-quantization_amd/csrc"
name=$1; flags=$2; src=${3:-pq_encode_cs.hip}
make -s -j8 >/dev/null
mkdir -p ../lib/ab/obj_$name
HIPFLAGS="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -ffp-contract=off -Wall -Wno-unused-function -fvisibility=hidden -fno-gpu-rdc -fno-slp-vectorize"
/opt/rocm/bin/hipcc $HIPFLAGS $flags -c $src -o ../lib/ab/obj_$name/${src%.hip}.o
objs=""
for o in ../lib/obj/*.o; do
  b=$(basename $o)
  if [ "$b" = "${src%.hip}.o" ]; then objs="$objs ../lib/ab/obj_$name/$b"; else objs="$objs $o"; fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../lib/ab/libmivq_$name.so $objs
rm -rf ../lib/ab/obj_$name
echo "built lib/ab/libmivq_$name.so"
