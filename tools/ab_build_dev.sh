#!/bin/bash
# tools/ab_build_dev.sh NAME "FLAGS": like ab_build.sh, but -mllvm options reach only the HIP translation unit (device code generation experiments)
# (A/B timing with SDFGEN_LIB_OVERRIDE=ab/NAME.so; diagnostics only).
set -e
cd "$(dirname "$0")/.."
mkdir -p ab/build_$1
H=/opt/rocm/bin/hipcc
F="-O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -fno-slp-vectorize -Iinclude -Isdfgenfast_amd/csrc $2"
$H --offload-arch=gfx950 $F -c sdfgenfast_amd/csrc/sdfgen_hip.hip -o ab/build_$1/a.o
$H -x hip --offload-arch=gfx950 $(echo $F | sed "s#-mllvm [^ ]*##g") -c sdfgenfast_amd/csrc/cpu_backend.cpp -o ab/build_$1/b.o
$H $(echo $F | sed "s#-mllvm [^ ]*##g") -c sdfgenfast_amd/csrc/sdfgen_unified.cpp -o ab/build_$1/c.o
$H $(echo $F | sed "s#-mllvm [^ ]*##g") -c sdfgenfast_amd/csrc/meshio.cpp -o ab/build_$1/d.o
$H -O2 -std=c++17 -fPIC -Iinclude -DSDFGEN_BUILD_ID="\"ab-$1\"" -c sdfgenfast_amd/csrc/build_id.cpp -o ab/build_$1/e.o
$H --offload-arch=gfx950 -shared -fPIC -o ab/$1.so ab/build_$1/*.o -lpthread
