#!/bin/bash
# Rehearsals of bench.py's N-rank paths on ONE GPU.  The in-launch exchange needs every rank's launch resident at
# once (and each launch its whole grid), which one GPU gives for 2 ranks; 8 ranks rehearse the RCCL-path logic
# (gloo all-gather + merge launch) with config 5's 8-way shards (a quad per sample).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3d; mkdir -p $O
run() { local n=$1; shift; timeout -k 10 400 python bench.py "$@" > $O/$n.json 2> $O/$n.err; local rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ] || { grep -E "Error|error" $O/$n.err | head -5; exit $rc; }
  python -c "import json;d=json.load(open('$O/$n.json'));print('  ranks', d['ranks'], 'n_gpus', d['n_gpus'], 'seen', d['ranks_seen'], 'exchange', d['config']['exchange'], 'lps', d['config']['lanes_per_sample'], 'K/GPU', d['config']['K_per_gpu'], 'ms/step %.4f'%d['ms_per_step'])"; }
run c3_2ranks_launch --gpus 2 --steps 500 --warmup 20 --cpu-seconds 0
run c5_2ranks_launch --gpus 2 --workload c5 --steps 100 --warmup 10 --cpu-seconds 0
run c5_8ranks_rccl --gpus 8 --workload c5 --exchange rccl --steps 50 --warmup 5 --cpu-seconds 0
run c3_8ranks_rccl --gpus 8 --exchange rccl --steps 100 --warmup 5 --cpu-seconds 0
