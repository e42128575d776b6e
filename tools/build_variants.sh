#!/bin/bash
# Diagnostic variants of the HIP library (never the product).  Outputs under
# mppi_robotarm_amd/_lib/libmppi_rocm_<name>.so.  Usage: build_variants.sh name:"-DFLAGS" ...
set -e
cd "$(dirname "$0")/.."
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  python3 -c "import sys; from mppi_robotarm_amd.build import build_native; build_native(True, sys.argv[1].split(), sys.argv[2])" \
    "$flags" "mppi_robotarm_amd/_lib/libmppi_rocm_$name.so" &
done
wait
