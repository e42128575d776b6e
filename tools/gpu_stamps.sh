#!/bin/bash
# GPU box: stamp timelines (diagnostic build) of the converged device loop at
# c3, c2 and c5.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/stamps; mkdir -p $O
L=mppi_robotarm_amd/_lib/libmppi_rocm_stamp.so
WARM=30 timeout -k 10 120 python tools/stamps.py $L 65536 64 4 > $O/c3.log 2>&1 || { tail $O/c3.log; exit 1; }
WARM=30 timeout -k 10 120 python tools/stamps.py $L 4096 32 4 > $O/c2.log 2>&1 || { tail $O/c2.log; exit 1; }
WARM=10 WORKLOAD=c5 timeout -k 10 120 python tools/stamps.py $L 131072 128 3 > $O/c5.log 2>&1 || { tail $O/c5.log; exit 1; }
tail -6 $O/c3.log; tail -6 $O/c2.log; tail -5 $O/c5.log
WARM=10 LPS=4 WORKLOAD=c5 timeout -k 10 120 python tools/stamps.py $L 16384 128 3 > $O/c5k16384.log 2>&1 || { tail $O/c5k16384.log; exit 1; }
tail -5 $O/c5k16384.log
