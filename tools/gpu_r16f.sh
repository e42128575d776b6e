#!/bin/bash
# round 6: the device NumPy draw — draw + host RNG tests, the draw's timing, kernel stats at P = 128 and 256.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r16f}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_npdraw.py tests/test_hostrng.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $O/tests.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/npdraw_bench.py > $O/bench.txt 2>&1
rc=$?; echo "bench rc=$rc"; grep -E "draw K|device draw\)" $O/bench.txt; [ $rc -eq 0 ] || exit $rc
for P in 128 256; do
  MPPI_NP_STRIDE=$P timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$P -o run -- python tools/npdraw_bench.py 65536 64 > $O/prof_$P.log 2>&1
  rc=$?; echo "prof P=$P rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
