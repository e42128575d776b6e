#!/bin/bash
# GPU box: the -m gpu suite on the product build, then tools/ab.py of
# libmppi_rocm_base.so (a saved earlier build) against the product at c3 and c2.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=mppi_robotarm_amd/_lib
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rf > gpurun_out/gputest.log 2>&1
rc=$?; echo "gputest rc=$rc"; tail -3 gpurun_out/gputest.log; [ $rc -eq 0 ] || { tail -60 gpurun_out/gputest.log; exit $rc; }
timeout -k 10 300 python tools/ab.py $L/libmppi_rocm_${AB_BASE:-base}.so $L/libmppi_rocm.so "$@" > gpurun_out/ab_c3.log 2>&1 || exit $?
timeout -k 10 300 python tools/ab.py $L/libmppi_rocm_${AB_BASE:-base}.so $L/libmppi_rocm.so "$@" 4096 32 > gpurun_out/ab_c2.log 2>&1 || exit $?
cat gpurun_out/ab_c3.log gpurun_out/ab_c2.log
