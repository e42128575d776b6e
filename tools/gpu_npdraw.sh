#!/bin/bash
# GPU box: the device NumPy-draw tests, its timing (the stride the plan picks, then forced strides), and a
# rocprofv3 kernel-trace of the timing run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-npdraw}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_npdraw.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/npdraw_bench.py > $O/bench.txt 2>&1
rc=$?; echo "bench rc=$rc"; cat $O/bench.txt; [ $rc -eq 0 ] || exit $rc
for P in ${STRIDES:-128 256 512}; do
  MPPI_NP_STRIDE=$P timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$P -o run -- python tools/npdraw_bench.py 65536 64 > $O/prof_$P.log 2>&1
  rc=$?; echo "prof P=$P rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
exit 0
