#!/usr/bin/env bash
# Build a variant of libkanode.so with kan_pp.hip compiled under extra macros (A/B experiments):
#   tools/build_var.sh NAME "-DKAN_PP_CHUNK=8 ..."   -> tools/bin/var/NAME.so
set -eu
cd "$(dirname "$0")/.."
name=$1; flags=$2
mkdir -p tools/bin/var/obj_$name
H="/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -Iinclude -Ikan-odes_amd/csrc"
$H $flags -c -o tools/bin/var/obj_$name/kan_pp.o kan-odes_amd/csrc/kan_pp.hip
objs=$(ls kan-odes_amd/build/*.o | grep -v kan_pp.o)
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o tools/bin/var/$name.so tools/bin/var/obj_$name/kan_pp.o $objs
echo built tools/bin/var/$name.so
