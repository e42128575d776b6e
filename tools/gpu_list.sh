#!/bin/bash
# GPU box: the chain's list-only rows — the chain and exchange GPU tests on the product, the chain tests on builds
# that make every eligible row list-only (the merger's own gathers) with the direct merge and with the group
# merges, one-process A/B at the c5 shard and K = 32768 (every-row-gathers build first), then the shard's
# profile (traffic).  Usage: gpu_list.sh OUT
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_exchange_world.py tests/test_gpu_exchange.py -x -q \
  --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $O/tests.log)"; [ $rc -eq 0 ] || { grep -E "^FAILED|^E " $O/tests.log | head -30; exit $rc; }
for v in pred0 pred0d0; do
  MPPI_LIB_PATH=$PWD/mppi_robotarm_amd/_lib/libmppi_rocm_$v.so timeout -k 10 600 python -u -m pytest \
    tests/test_gpu_chain.py -x -q --timeout 300 --timeout-method thread > $O/$v.log 2>&1
  rc=$?; echo "$v rc=$rc $(tail -1 $O/$v.log)"; [ $rc -eq 0 ] || { grep -E "^FAILED|^E " $O/$v.log | head -30; exit $rc; }
done
AB_K="16384 32768" bash tools/gpu_q4ab.sh $1/ab libmppi_rocm_nolist.so libmppi_rocm.so libmppi_rocm_pred0.so || exit $?
bash tools/profile_round.sh $1 c5 "--K 16384" || exit $?
