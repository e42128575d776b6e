#!/bin/bash
# GPU box: the -m gpu suite (achieved parity numbers recorded to parity_records.jsonl),
# smoke(), and the c3 and c2 bench lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/check; mkdir -p $O
rm -f $O/parity_records.jsonl
export MPPI_PARITY_RECORD=$PWD/$O/parity_records.jsonl
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=5 --timeout 300 --timeout-method thread -rf -s > $O/gputest.log 2>&1
rc=$?; echo "gputest rc=$rc"; grep -E "passed|failed" $O/gputest.log | tail -3; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/gputest.log | head -40; exit $rc; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
echo smoke ok
for W in c3 c2; do
  timeout -k 10 300 python bench.py --workload $W > $O/bench_$W.json 2> $O/bench_$W.err || { tail -30 $O/bench_$W.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_$W.json'));print('$W', 'kernel_us', round(d['kernel_ms']*1e3,2), 'ms_per_step', round(d['ms_per_step'],4), 'lat_ms', d['control_step_latency_ms'], 'b2b', d.get('control_step_latency_back_to_back_ms'), 'frac', round(d['roofline']['frac'],4), 'lps', d['config']['lanes_per_sample'])"
done
