#!/usr/bin/env bash
# Build a variant of libkanode.so with some sources compiled under extra macros (A/B experiments):
#   tools/build_var.sh NAME "-DKAN_PP_CHUNK=8 ..." [sources, default kan_pp.hip]  -> tools/bin/var/NAME.so
set -eu
cd "$(dirname "$0")/.."
name=$1; flags=$2; shift 2
srcs=${*:-kan_pp.hip}
mkdir -p tools/bin/var/obj_$name
H="/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -Iinclude -Ikan-odes_amd/csrc"
objs=""
for f in kan-odes_amd/build/*.o; do
  b=$(basename $f .o)
  hit=""
  for s in $srcs; do [ "${s%.*}" = "$b" ] && hit=$s; done
  if [ -n "$hit" ]; then
    case $hit in *.cpp) X="-x hip";; *) X="";; esac
    $H $X $flags -c -o tools/bin/var/obj_$name/$b.o kan-odes_amd/csrc/$hit
    objs="$objs tools/bin/var/obj_$name/$b.o"
  else
    objs="$objs $f"
  fi
done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o tools/bin/var/$name.so $objs -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo built tools/bin/var/$name.so
