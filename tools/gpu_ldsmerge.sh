#!/bin/bash
# Whole-row LDS merge: the 2-DoF GPU parity suite (hand-off forms bit-identical, shards, fixtures), then
# one-process A/B against the previous build at c2 and c3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/ldsm; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_exchange.py tests/test_gpu_multigpu_dropin.py -q --timeout 300 --timeout-method thread -rf > $O/parity.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -3 $O/parity.log; [ $rc -le 1 ] || exit $rc
[ $rc -eq 0 ] || { grep -E "^FAILED|^E " $O/parity.log | head -20; exit 1; }
B=mppi_robotarm_amd/_lib/libmppi_rocm_base.so; P=mppi_robotarm_amd/_lib/libmppi_rocm.so
timeout -k 10 300 python tools/ab.py $B $P 4096 32 40 50 > $O/ab_c2.txt 2>&1 || exit 1
timeout -k 10 300 python tools/ab.py $B $P 65536 64 30 50 > $O/ab_c3.txt 2>&1 || exit 1
grep -E "median|K=" $O/ab_c2.txt $O/ab_c3.txt
