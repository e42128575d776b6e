#!/bin/bash
# sampled_traj_list through the chunked fp32 read-back widened on host threads: its GPU tests, the sampled
# parity tests, tools/sampled_latency.py (both legs, the route comparison and the worker/chunk sweep).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/sampled; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_readback.py tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "readback or sampled or runpy_k100" > $O/gputest.log 2>&1
rc=$?; echo "gputest rc=$rc"; grep -E "passed|failed" $O/gputest.log | tail -3; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/gputest.log | head -40; exit $rc; }
timeout -k 10 400 python -u tools/sampled_latency.py ${1:-} > $O/sampled_latency.txt 2>&1 || { tail -20 $O/sampled_latency.txt; exit 1; }
grep -v amdgpu.ids $O/sampled_latency.txt
