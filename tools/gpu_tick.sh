#!/bin/bash
# Drop-in tick: its GPU tests, the latency breakdown and the c3 bench line's latency fields.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/tick; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 120 --timeout-method thread \
    -k "tick or sigma or dropin or close" > $O/gputest.log 2>&1
rc=$?; echo "gputest rc=$rc"; grep -E "passed|failed" $O/gputest.log | tail -2; [ $rc -eq 0 ] || { grep -E "^FAILED|^E " $O/gputest.log | head -20; exit $rc; }
timeout -k 10 300 python tools/latency_breakdown.py > $O/latency_breakdown.txt 2>&1 || { tail -5 $O/latency_breakdown.txt; exit 1; }
cat $O/latency_breakdown.txt
timeout -k 10 300 python bench.py --cpu-seconds 0 > $O/c3.json 2> $O/c3.err || { tail -5 $O/c3.err; exit 1; }
python -c "import json;d=json.load(open('$O/c3.json'));print('c3 kernel_us', round(d['kernel_ms']*1e3,2), 'lat', round(d['control_step_latency_ms'],4), 'p90', round(d['control_step_latency_p90_ms'],4), 'b2b', round(d['control_step_latency_back_to_back_ms'],4))"
