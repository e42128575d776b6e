#!/bin/bash
# Endurance (tools/stress.py: c3, c5, c5 shard), then 8-rank rehearsals of bench.py on ONE GPU (gloo for the
# setup collectives, the in-launch exchange between 8 same-device inboxes): c3 weak scaling and c5 strong
# scaling (8 shards of 16384 samples, a quad per sample).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3c; mkdir -p $O
timeout -k 10 300 python tools/stress.py > $O/stress.txt 2>&1; rc=$?; echo "stress rc=$rc"; grep -v amdgpu.ids $O/stress.txt | tail -4; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --gpus 8 --steps 300 --warmup 20 --cpu-seconds 0 > $O/bench_8ranks_c3.json 2> $O/bench_8ranks_c3.err; rc=$?; echo "8 ranks c3 rc=$rc"; [ $rc -eq 0 ] || { tail -20 $O/bench_8ranks_c3.err; exit $rc; }
timeout -k 10 400 python bench.py --gpus 8 --workload c5 --steps 100 --warmup 10 --cpu-seconds 0 > $O/bench_8ranks_c5.json 2> $O/bench_8ranks_c5.err; rc=$?; echo "8 ranks c5 rc=$rc"; [ $rc -eq 0 ] || { tail -20 $O/bench_8ranks_c5.err; exit $rc; }
for f in c3 c5; do python -c "import json;d=json.load(open('$O/bench_8ranks_$f.json'));print('$f', 'ranks', d['ranks'], 'n_gpus', d['n_gpus'], 'seen', d['ranks_seen'], 'exchange', d['config']['exchange'], 'lps', d['config']['lanes_per_sample'], 'ms/step %.4f'%d['ms_per_step'])"; done
