#!/bin/bash
# sampled_traj_list through the pinned read-back pool: the -m gpu suite, tools/sampled_latency.py, the c3 bench
# line (control_step_latency_sampled_trajs_ms).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/sampled; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=5 --timeout 300 --timeout-method thread -rf > $O/gputest.log 2>&1
rc=$?; echo "gputest rc=$rc"; grep -E "passed|failed" $O/gputest.log | tail -3; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/gputest.log | head -40; exit $rc; }
timeout -k 10 300 python tools/sampled_latency.py > $O/sampled_latency.txt 2>&1 || { tail -20 $O/sampled_latency.txt; exit 1; }
grep -v amdgpu.ids $O/sampled_latency.txt
timeout -k 10 300 python bench.py --workload c3 > $O/bench_c3.json 2> $O/bench_c3.err || { tail -30 $O/bench_c3.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_c3.json'));print({k: v for k, v in d.items() if 'latency' in k and 'def' not in k})"
