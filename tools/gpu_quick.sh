#!/bin/bash
# The -m gpu suite, then the c3 bench line (drop-in latency fields) without the CPU baseline.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/quick; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=5 --timeout 300 --timeout-method thread -rf > $O/gputest.log 2>&1
rc=$?; echo "gputest rc=$rc"; grep -E "passed|failed" $O/gputest.log | tail -2; [ $rc -le 1 ] || exit $rc
[ $rc -eq 0 ] || grep -E "^FAILED|^E " $O/gputest.log | head -20
timeout -k 10 300 python bench.py --cpu-seconds 0 > $O/c3.json 2> $O/c3.err || { tail -5 $O/c3.err; exit 1; }
python -c "import json;d=json.load(open('$O/c3.json'));print('c3 kernel_us', round(d['kernel_ms']*1e3,2), 'lat', round(d['control_step_latency_ms'],4), 'p90', round(d['control_step_latency_p90_ms'],4), 'b2b', round(d['control_step_latency_back_to_back_ms'],4))"
