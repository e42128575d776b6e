#!/bin/bash
# GPU box: the device NumPy-draw tests, its timing, and a rocprofv3 kernel-trace of the timing run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-npdraw}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_npdraw.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python tools/npdraw_bench.py > $O/bench.txt 2>&1
rc=$?; echo "bench rc=$rc"; cat $O/bench.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python tools/npdraw_bench.py > $O/prof.log 2>&1
rc=$?; echo "prof rc=$rc"
exit 0
