#!/bin/bash
# Config 5 bench lines: fp32 and fp64 rollout at K = 131072, and the 8-way shard proxy K = 16384 (fp32).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/c5; mkdir -p $O
for cfg in "f32 131072" "f64 131072" "f32 16384"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --workload c5 --precision $1 --K $2 --cpu-seconds 0 > $O/bench_$1_$2.json 2> $O/bench_$1_$2.err || { tail -5 $O/bench_$1_$2.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_$1_$2.json'));print('c5 $1 K=$2', 'kernel_us', round(d['kernel_ms']*1e3,2), 'ms_per_step', round(d['ms_per_step'],4))"
done
