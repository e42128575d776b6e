#!/bin/bash
# GPU box: lanes-per-sample sweep at small K (one-process A/B of LPS 2/4/8 on
# the product build), for auto_lps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/lps; mkdir -p $O
L=mppi_robotarm_amd/_lib/libmppi_rocm.so
for KT in "2048 32" "4096 32" "4096 64" "8192 32" "8192 64" "16384 64" "32768 64"; do
  LPS_LIST=2,4,8 timeout -k 10 120 python tools/ab.py $L $L $L $KT > $O/ab_${KT// /_}.log 2>&1 || { cat $O/ab_${KT// /_}.log; exit 1; }
  grep -h "median\|K=" $O/ab_${KT// /_}.log
done
