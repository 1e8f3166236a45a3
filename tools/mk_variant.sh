#!/bin/bash
# Links an alternative library ldpc_sparc_amd/_lib_v_<name>/ from the current
# objects with one source recompiled under extra flags, for tools/ab_multi.sh:
#   tools/mk_variant.sh <name> <source.hip> <flags...>
set -e
cd "$(dirname "$0")/.."
name=$1; src=$2; shift 2
C=ldpc_sparc_amd/csrc; O=ldpc_sparc_amd/_lib/obj; D=ldpc_sparc_amd/_lib_v_$name
mkdir -p $D/obj
base=$(basename $(basename $src .hip) .cpp)
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -Wno-unused-value --offload-arch=gfx950 \
  -Iinclude "$@" -x hip -c $C/$src -o $D/obj/$base.o
objs=$(ls $O/*.o | grep -v "/$base.o$")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $D/libldpc_sparc_amd.so $objs $D/obj/$base.o -lrccl
rm -rf $D/obj
echo "built $D"
