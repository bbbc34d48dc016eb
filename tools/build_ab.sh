#!/bin/bash
# A/B library variant: $SRC (default np_sampler.hip) rebuilt with extra flags, linked with the product objects
# into lib_ab/<name>/librsamd.so (use with RSAMD_LIB).  Usage: bash tools/build_ab.sh <name> <flags...>
set -e
NAME=$1; shift
C=$(cd "$(dirname "$0")/../tsbb15-3d-reconstruction-project_amd/csrc" && pwd)
make -C $C -s
B=$C/build_ab_$NAME; mkdir -p $B
cp $C/build/*.o $B/
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -fno-slp-vectorize -I$C/../../include -Wall "$@" -c $C/${SRC:-np_sampler.hip} -o $B/$(basename ${SRC:-np_sampler.hip} .hip).o
mkdir -p $C/../lib_ab/$NAME
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $C/../lib_ab/$NAME/librsamd.so $B/*.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo built $C/../lib_ab/$NAME/librsamd.so
