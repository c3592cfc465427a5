#!/bin/bash
# Build libgvl_<name>.so: the shipped objects with ONE source recompiled under extra -D flags
# (A/B of compile-time kernel variants; load it with GVL_LIB=...).
# usage: tools/r3/build_variant.sh name source.hip "-DFOO=1 ..."
set -e
R=$(cd "$(dirname "$0")/../.." && pwd)
NAME=$1; SRC=$2; FLAGS=$3
C=$R/gpt2-vision-language_amd/csrc; B=$R/build/gvl; V=$R/build/var_$NAME
mkdir -p $V
make -C $C -j8 > /dev/null
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function \
  -mllvm -pragma-unroll-threshold=1000000 $FLAGS -c $C/$SRC -o $V/${SRC%.hip}.o
OBJS=$(ls $B/*.o | grep -v "/${SRC%.hip}.o$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $R/gpt2-vision-language_amd/gvl/libgvl_$NAME.so $OBJS $V/${SRC%.hip}.o
echo built libgvl_$NAME.so
