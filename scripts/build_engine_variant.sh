#!/bin/bash
# A/B builds of the engine: compiles device_engine.hip (optionally from another source tree,
# SRC_DIR) with extra defines and links it with the release objects into
# libfst_amd/variants/<name>.so (select with LIBFST_AMD_LIB=...).
# usage: [SRC_DIR=dir] scripts/build_engine_variant.sh <name> "<-DFLAG ...>"
set -e
cd "$(dirname "$0")/../libfst_amd/csrc"
[ -n "$SKIP_MAKE" ] || make -s -j8
name=$1; defs=$2
src=${SRC_DIR:-.}
vdir=${VARIANT_DIR:-../variants}
mkdir -p $vdir build_var
HIPCC=/opt/rocm/bin/hipcc
$HIPCC -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -ffp-contract=off $defs --offload-arch=gfx950 \
  -I. -c $src/device_engine.hip -o build_var/de_$name.o
$HIPCC -shared -fPIC --offload-arch=gfx950 -o $vdir/$name.so \
  build/host_fst.cpp.o build/c_api.cpp.o build_var/de_$name.o build/eager_pull.hip.o
echo "built $vdir/$name.so ($defs)"
