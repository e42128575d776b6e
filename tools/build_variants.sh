#!/bin/bash
# Diagnostic variants of the HIP library (never the product).  Outputs under
# mppi_robotarm_amd/_lib/libmppi_rocm_<name>.so.  Usage: build_variants.sh name:"-DFLAGS" ...
set -e
cd "$(dirname "$0")/.."
SRC=mppi_robotarm_amd/csrc/mppi_rocm.hip
OUT=mppi_robotarm_amd/_lib
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Iinclude"
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  hipcc $F $flags -o $OUT/libmppi_rocm_$name.so $SRC &
done
wait
