#!/bin/bash
# GPU box: the -m gpu suite, smoke(), and the bench lines: c3 (with the drop-in latencies), c2, c5, c5 at its
# 8-way shard size (K = 16384), and a 2-rank rehearsal of c3 on the one GPU (in-launch exchange).
# Usage: gpu_full.sh OUT [skip-tests]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-full}; mkdir -p $O
export MPPI_PARITY_RECORD=$PWD/$O/parity_records.jsonl
if [ "${2:-}" != "skip-tests" ]; then
  rm -f $MPPI_PARITY_RECORD
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=5 --timeout 300 --timeout-method thread -rf -s > $O/gputest.log 2>&1
  rc=$?; echo "gputest rc=$rc"; grep -E "passed|failed" $O/gputest.log | tail -2; [ $rc -eq 0 ] || { grep -E "^FAILED|^E " $O/gputest.log | head -40; exit $rc; }
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
  echo smoke ok
fi
summ() { python -c "import json,sys;d=json.load(open('$1'));print('$2', 'kernel_us', round(d['kernel_ms']*1e3,2), 'ms_per_step', round(d['ms_per_step'],4), 'frac', round(d['roofline']['frac'],4), 'lat', d.get('control_step_latency_ms'), 'b2b', d.get('control_step_latency_back_to_back_ms'), 'np', d.get('control_step_latency_numpy_noise_ms'), 'lps', d['config'].get('lanes_per_sample'), 'x', d['config'].get('exchange'))"; }
for W in "c3" "c2" "c5" "c5 --K 16384"; do
  n=$(echo $W | tr ' ' '_' | tr -d '-')
  timeout -k 10 300 python bench.py --workload $W > $O/bench_$n.json 2> $O/bench_$n.err || { tail -30 $O/bench_$n.err; exit 1; }
  summ $O/bench_$n.json "$n"
done
timeout -k 10 300 python bench.py --gpus 2 --steps 2000 --cpu-seconds 0 > $O/bench_c3_2ranks.json 2> $O/bench_c3_2ranks.err || { tail -30 $O/bench_c3_2ranks.err; exit 1; }
summ $O/bench_c3_2ranks.json c3_2ranks
