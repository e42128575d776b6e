#!/bin/bash
# Chain GPU tests first (fp64 rollout, spread weights, tie-explained outliers), then gpu_check.sh, then the c5
# bench lines for the fp32 and the fp64 rollout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/check; mkdir -p $O
export MPPI_PARITY_RECORD=$PWD/$O/parity_chain.jsonl
rm -f $MPPI_PARITY_RECORD
timeout -k 10 600 python -u -m pytest tests/test_gpu_chain.py -v --timeout 300 --timeout-method thread -rf -s > $O/chain.log 2>&1
rc=$?; echo "chain rc=$rc"; grep -E "passed|failed" $O/chain.log | tail -2; [ $rc -le 1 ] || exit $rc
[ $rc -eq 0 ] || { grep -E "^FAILED|^E " $O/chain.log | head -30; exit 1; }
bash tools/gpu_check.sh; rc=$?; [ $rc -le 1 ] || exit $rc
for P in f32 f64; do
  timeout -k 10 300 python bench.py --workload c5 --precision $P --cpu-seconds 0 > $O/bench_c5_$P.json 2> $O/bench_c5_$P.err || { tail -5 $O/bench_c5_$P.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_c5_$P.json'));print('c5 $P', 'kernel_us', round(d['kernel_ms']*1e3,2), 'ms_per_step', round(d['ms_per_step'],4))"
done
