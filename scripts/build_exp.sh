#!/bin/bash
# Experiment builds of libgpumatch.so with extra -D flags (measurement only, never shipped):
#   scripts/build_exp.sh NAME "-DFLAG ..."   ->  exp/NAME/libgpumatch.so  (load with GM_LIB=...)
set -e
cd "$(dirname "$0")/../ingress-plus_amd/csrc"
make -s ../libgpumatch.so
out=../../exp/$1
mkdir -p "$out"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -Wno-unused-variable $2 --offload-arch=gfx950 -c gm_device.hip -o "$out/gm_device.o"
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$out/libgpumatch.so" "$out/gm_device.o" gm_compile.o gm_regex.o -L/opt/rocm/lib -lrccl -lamdhip64
rm -f "$out/gm_device.o"
