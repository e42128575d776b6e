#!/bin/bash
# The chain in absolute angles: the chain parity tests, then the one-process A/B against the joint-angle
# build (libmppi_rocm_qspace.so) at config 5.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/theta; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_exchange.py -q -x --timeout 300 --timeout-method thread -m gpu > $O/test.log 2>&1
rc=$?; tail -3 $O/test.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $O/test.log | head -20; exit $rc; }
WORKLOAD=c5 timeout -k 10 300 python tools/ab.py mppi_robotarm_amd/_lib/libmppi_rocm_qspace.so mppi_robotarm_amd/_lib/libmppi_rocm.so 131072 128 20 20 > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
cat $O/ab.log
