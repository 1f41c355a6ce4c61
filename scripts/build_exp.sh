#!/bin/bash
# Experiment builds of libgpumatch.so with extra -D flags (measurement only, never shipped):
#   scripts/build_exp.sh NAME "-DFLAG ..."   ->  exp/NAME/libgpumatch.so  (load with GM_LIB=...)
set -e
cd "$(dirname "$0")/../ingress-plus_amd/csrc"
make -s ../libgpumatch.so
out=../../exp/$1
mkdir -p "$out"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -Wno-unused-variable $2 --offload-arch=gfx950 -c gm_device.hip -o "$out/gm_device.o"
# EXP_HOST=1: the host objects too (flags that change the table image, e.g. GM_SCAN_HASH2)
objs="gm_compile.o gm_regex.o gm_buildid.o"
if [ -n "$EXP_HOST" ]; then
  for f in gm_compile gm_regex; do
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -Wno-unused-variable $2 -x c++ -c $f.cpp -o "$out/$f.o" &
  done
  wait
  objs="$out/gm_compile.o $out/gm_regex.o gm_buildid.o"
fi
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$out/libgpumatch.so" "$out/gm_device.o" $objs -L/opt/rocm/lib -lrccl -lamdhip64
rm -f "$out"/*.o
