#!/bin/bash
# GPU box: chain quad-per-sample variants at the c5 shard — the chain parity tests on each variant library,
# then one-process A/B timings (tools/ab.py).  Usage: gpu_q4ab.sh OUT lib1.so lib2.so ...  (first = baseline)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/$1; shift; mkdir -p $O
libs=""
for l in "$@"; do
  libs="$libs mppi_robotarm_amd/_lib/$l"
  [ "$l" = libmppi_rocm.so ] && continue
  MPPI_LIB_PATH=$PWD/mppi_robotarm_amd/_lib/$l timeout -k 10 600 python -u -m pytest tests/test_gpu_chain.py -x -q \
    --timeout 300 --timeout-method thread -k "n7 or every_link_count_against or short or lanes_per or fused" > $O/t_$l.log 2>&1
  rc=$?; echo "$l tests rc=$rc $(tail -1 $O/t_$l.log)"; [ $rc -eq 0 ] || { grep -E "^FAILED|^E " $O/t_$l.log | head -20; exit $rc; }
done
for K in ${AB_K:-16384}; do
  WORKLOAD=c5 timeout -k 10 400 python -u tools/ab.py $libs $K 128 12 20 > $O/ab_c5k$K.txt 2>&1 || { tail -20 $O/ab_c5k$K.txt; exit 1; }
  cat $O/ab_c5k$K.txt
done
