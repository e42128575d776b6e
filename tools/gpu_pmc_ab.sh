#!/bin/bash
# SQ counter passes of the rollout kernel for two library builds (diagnostic).
# Usage: tools/gpu_pmc_ab.sh VARIANT_A VARIANT_B   ("" = product)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for V in "$@"; do
  [ "$V" = prod ] && V=""
  LIB=$PWD/mppi_robotarm_amd/_lib/libmppi_rocm${V:+_$V}.so
  O=gpurun_out/pmcab_${V:-prod}; mkdir -p $O
  B="python3 bench.py --steps 20 --warmup 2 --settle-ms 0 --cpu-seconds 0"
  MPPI_LIB_PATH=$LIB timeout -k 10 120 rocprofv3 --kernel-include-regex rollout --output-format csv -d $O/p1 -o p \
    --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_BUSY_CYCLES \
    -- $B > $O/p1.log 2>&1 || { echo "pmc $V rc=$?"; exit 1; }
  MPPI_LIB_PATH=$LIB timeout -k 10 120 rocprofv3 --kernel-include-regex rollout --output-format csv -d $O/p2 -o p \
    --pmc SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_RD SQ_WAVES GRBM_GUI_ACTIVE \
    -- $B > $O/p2.log 2>&1 || { echo "pmc2 $V rc=$?"; exit 1; }
done
python3 - "$@" <<'PY'
import csv, glob, sys, collections
for V in sys.argv[1:]:
    d = collections.defaultdict(list)
    for f in glob.glob(f"gpurun_out/pmcab_{'prod' if V in ('', 'prod') else V}/p*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            d[r['Counter_Name']].append(float(r['Counter_Value']))
    print(V, {k: round(sum(v) / max(1, len(v))) for k, v in sorted(d.items())})
PY
