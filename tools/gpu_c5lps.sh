#!/bin/bash
# Chain lanes per sample: the chain GPU tests, then c5 bench lines at K = 16384 / 32768 / 65536 with one lane and
# a quad per sample (the table behind chain_auto_lps).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/c5lps; mkdir -p $O
export MPPI_PARITY_RECORD=$PWD/$O/parity_chain.jsonl
rm -f $MPPI_PARITY_RECORD
timeout -k 10 600 python -u -m pytest tests/test_gpu_chain.py -v --timeout 300 --timeout-method thread -rf -s > $O/chain.log 2>&1
rc=$?; echo "chain rc=$rc"; grep -E "passed|failed" $O/chain.log | tail -2; [ $rc -le 1 ] || exit $rc
[ $rc -eq 0 ] || { grep -E "^FAILED|^E " $O/chain.log | head -30; }
for K in 16384 32768 65536; do for L in 1 4; do
  timeout -k 10 300 python bench.py --workload c5 --K $K --lps $L --cpu-seconds 0 --steps 300 > $O/b_${K}_$L.json 2> $O/b_${K}_$L.err || { tail -5 $O/b_${K}_$L.err; exit 1; }
  python -c "import json;d=json.load(open('$O/b_${K}_$L.json'));print('c5 K=$K lps', d['config']['lanes_per_sample'], 'kernel_us', round(d['kernel_ms']*1e3,2))"
done; done
