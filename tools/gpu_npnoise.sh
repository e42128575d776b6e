#!/bin/bash
# The drop-in's default NumPy-stream noise through hostrng: the -m gpu suite, then tools/numpy_noise_latency.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/npnoise; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=5 --timeout 300 --timeout-method thread -rf > $O/gputest.log 2>&1
rc=$?; echo "gputest rc=$rc"; grep -E "passed|failed" $O/gputest.log | tail -3; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/gputest.log | head -40; exit $rc; }
timeout -k 10 300 python -m pytest tests/test_hostrng.py -q > $O/hostrng_test.log 2>&1 || { tail -20 $O/hostrng_test.log; exit 1; }
tail -1 $O/hostrng_test.log
timeout -k 10 300 python tools/numpy_noise_latency.py > $O/numpy_noise_latency.txt 2>&1 || { tail -20 $O/numpy_noise_latency.txt; exit 1; }
grep -v amdgpu.ids $O/numpy_noise_latency.txt
