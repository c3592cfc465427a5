#!/bin/bash
# Build libgvl_<name>.so: the shipped objects with SEVERAL sources recompiled under extra -D
# flags (A/B of compile-time kernel variants spanning files; load it with GVL_LIB=...).
# usage: tools/build_variant.sh name "-DFOO=1 ..." src1.hip src2.hip ...
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; FLAGS=$2; shift 2
C=$R/gpt2-vision-language_amd/csrc; B=$R/build/gvl; V=$R/build/var_$NAME
mkdir -p $V
make -C $C -j8 > /dev/null
pids=""
for SRC in "$@"; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function \
    -mllvm -pragma-unroll-threshold=1000000 $FLAGS -c $C/$SRC -o $V/${SRC%.hip}.o & pids="$pids $!"
done
for p in $pids; do wait $p; done
OBJS=""
for o in $B/*.o; do
  base=$(basename $o); [ -f $V/$base ] && OBJS="$OBJS $V/$base" || OBJS="$OBJS $o"
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $R/gpt2-vision-language_amd/gvl/libgvl_$NAME.so $OBJS
echo built libgvl_$NAME.so
