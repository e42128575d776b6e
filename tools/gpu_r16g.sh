#!/bin/bash
# round 6: the draw with the jump sequence read from the last draw's words — draw, multi-rank drop-in and host RNG
# tests, the NumPy-noise endurance run, and the draw's kernel stats at c3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r16l}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_npdraw.py tests/test_gpu_multigpu_dropin.py tests/test_hostrng.py -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $O/tests.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/np_endurance.py 300 > $O/endurance.txt 2>&1
rc=$?; tail -1 $O/endurance.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python tools/npdraw_bench.py > $O/prof.log 2>&1
rc=$?; grep -E "draw K|device draw\)" $O/prof.log; exit $rc
