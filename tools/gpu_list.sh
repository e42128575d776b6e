#!/bin/bash
# GPU box: the chain's list rows — the -m gpu suite on the product, the chain tests on a build whose merges
# always take the group rows (list rows in the group mergers), one-process A/B at the c5 shard and K = 32768
# (gather-everything build first), then the shard's profile (traffic).  Usage: gpu_list.sh OUT
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
rc=$?; echo "gputest rc=$rc $(tail -1 $O/gputest.log)"; [ $rc -eq 0 ] || { grep -E "^FAILED|^E " $O/gputest.log | head -30; exit $rc; }
MPPI_LIB_PATH=$PWD/mppi_robotarm_amd/_lib/libmppi_rocm_direct0.so timeout -k 10 600 python -u -m pytest \
  tests/test_gpu_chain.py -x -q --timeout 300 --timeout-method thread > $O/direct0.log 2>&1
rc=$?; echo "direct0 rc=$rc $(tail -1 $O/direct0.log)"; [ $rc -eq 0 ] || { grep -E "^FAILED|^E " $O/direct0.log | head -30; exit $rc; }
AB_K="16384 32768" bash tools/gpu_q4ab.sh $1/ab libmppi_rocm_nolist.so libmppi_rocm.so libmppi_rocm_list4.so || exit $?
bash tools/profile_round.sh $1 c5 "--K 16384" || exit $?
