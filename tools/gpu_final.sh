#!/bin/bash
# The whole -m gpu suite, smoke, and every bench line (c3, c2, c5, c5 at the shard size, c5 fp64).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_check.sh || exit $?
O=gpurun_out/final; mkdir -p $O
timeout -k 10 400 python bench.py --workload c5 > $O/c5.json 2> $O/c5.err || { tail -20 $O/c5.err; exit 1; }
timeout -k 10 400 python bench.py --workload c5 --K 16384 --cpu-seconds 0 > $O/c5_k16384.json 2> $O/c5_k16384.err || { tail -20 $O/c5_k16384.err; exit 1; }
timeout -k 10 400 python bench.py --workload c5 --precision f64 --cpu-seconds 0 > $O/c5_f64.json 2> $O/c5_f64.err || { tail -20 $O/c5_f64.err; exit 1; }
for f in c5 c5_k16384 c5_f64; do
  python -c "import json;d=json.load(open('$O/$f.json'));print('$f', 'kernel_us', round(d['kernel_ms']*1e3,2), 'value', '%.3g' % d['value'], 'b2b_ms', d.get('control_step_latency_back_to_back_ms'), 'lps', d['config'].get('lanes_per_sample'))"
done
