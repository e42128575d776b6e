#!/bin/bash
# Chain parity with the device's own window picks (mppi_chain_debug_slots), achieved numbers recorded.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/slots; mkdir -p $O
rm -f $O/records.jsonl
export MPPI_PARITY_RECORD=$PWD/$O/records.jsonl
timeout -k 10 600 python -u -m pytest tests/test_gpu_chain.py -v -s --timeout 300 --timeout-method thread -rf -k "n7_against" > $O/test.log 2>&1
rc=$?; grep -E "passed|failed" $O/test.log | tail -2; grep -E "beyond|picks" $O/test.log | head -20
[ $rc -eq 0 ] || { grep -E "^E |FAILED" $O/test.log | head -30; exit $rc; }
cat $O/records.jsonl
