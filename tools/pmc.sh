#!/bin/bash
# PMC counter passes (one counter set per pass) of the rollout kernel for one
# library variant.  Usage: tools/pmc.sh VARIANT   (libmppi_rocm_VARIANT.so; "" = product)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
V=${1:-}
LIB=$PWD/mppi_robotarm_amd/_lib/libmppi_rocm${V:+_$V}.so
export MPPI_LIB_PATH=$LIB
O=gpurun_out/pmc_${V:-prod}; mkdir -p $O
B="python3 bench.py --steps 20 --warmup 2 --cpu-seconds 0"
run() { local n=$1; shift; timeout -k 10 300 rocprofv3 --kernel-include-regex rollout --output-format csv -d $O/$n -o p "$@" -- $B > $O/$n.log 2>&1; local rc=$?; echo "$n rc=$rc"; [ $rc -le 1 ] || exit $rc; }
run p1 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_BUSY_CYCLES
run p2 --pmc GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAVES SQ_INSTS_VMEM_RD
run p3 --pmc FETCH_SIZE
run p4 --pmc WRITE_SIZE
