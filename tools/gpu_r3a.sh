#!/bin/bash
# Round 3 first pass: the -m gpu suite + smoke + c3/c2 bench lines (gpu_check.sh), then the config-5
# diagnostics: spread-weight accuracy (c5_dense.py) and the 8-way shard proxy (K = 16384 per GPU).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/check; mkdir -p $O
bash tools/gpu_check.sh; rc=$?
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python tools/c5_dense.py > $O/c5_dense.txt 2>&1; rc=$?; echo "c5_dense rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload c5 --K 16384 --cpu-seconds 0 > $O/bench_c5_k16384.json 2> $O/bench_c5_k16384.err; rc=$?
echo "c5 proxy rc=$rc"; cat $O/bench_c5_k16384.json | cut -c1-400
