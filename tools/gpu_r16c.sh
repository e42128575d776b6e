#!/bin/bash
# round 6: the multi-GPU diagnostics rehearsed on one GPU — exchange tests, bench.py --gpus 8 --K 1536 and
# --gpus 2 (c3) lines with exchange_selfcheck / exchange_costs / ranks_seen.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r16c; mkdir -p $O
fatal() { case $1 in 124|137|134|139) echo "fatal rc $1 in $2: stopping"; exit "$1";; esac; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_exchange_world.py tests/test_gpu_multigpu_dropin.py tests/test_gpu_exchange.py -q --timeout 120 --timeout-method thread > $O/xtests.log 2>&1
rc=$?; echo "exchange tests rc=$rc"; tail -2 $O/xtests.log; fatal $rc xtests; [ $rc -eq 0 ] || exit $rc
GPU_MAX_HW_QUEUES=1 timeout -k 10 300 python bench.py --gpus 8 --K 1536 --lps 1 --steps 500 --warmup 20 --cpu-seconds 0 > $O/bench_w8_k1536.json 2> $O/bench_w8_k1536.err
rc=$?; echo "bench w8 rc=$rc"; fatal $rc bench_w8; [ $rc -eq 0 ] || { tail -20 $O/bench_w8_k1536.err; exit $rc; }
timeout -k 10 300 python bench.py --gpus 2 --steps 2000 --cpu-seconds 0 > $O/bench_c3_2ranks.json 2> $O/bench_c3_2ranks.err
rc=$?; echo "bench c3 2 ranks rc=$rc"; fatal $rc bench_2; [ $rc -eq 0 ] || { tail -20 $O/bench_c3_2ranks.err; exit $rc; }
for f in $O/bench_w8_k1536.json $O/bench_c3_2ranks.json; do python -c "
import json; d = json.load(open('$f'))
print('$f', {k: d[k] for k in ('n_gpus', 'ranks', 'ranks_seen', 'ms_per_step', 'exchange_selfcheck', 'exchange_costs')})"; done
