#!/bin/bash
# Box-Muller with the constant folded into the Cholesky factor: the noise-stream tests, then the
# Philox draw A/B against the previous build (libmppi_rocm_bmold.so) in one process.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/bm; mkdir -p $O
rm -f $O/records.jsonl
export MPPI_PARITY_RECORD=$PWD/$O/records.jsonl
timeout -k 10 300 python -u -m pytest tests/test_gpu_noise_stream.py -v --timeout 240 --timeout-method thread -rf > $O/test.log 2>&1
rc=$?; grep -E "passed|failed" $O/test.log | tail -2; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/test.log | head -30; exit $rc; }
cat $O/records.jsonl
WORKLOAD=philox timeout -k 10 120 python tools/ab.py mppi_robotarm_amd/_lib/libmppi_rocm_bmold.so mppi_robotarm_amd/_lib/libmppi_rocm.so 65536 64 30 50 > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
cat $O/ab.log
