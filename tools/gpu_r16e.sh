#!/bin/bash
# round 6: the device NumPy draw after the twist / jump / host-mapped result changes — draw tests, the draw
# timing, kernel stats, and one SQ counter pass over the draw's kernels.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r16e}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_npdraw.py tests/test_hostrng.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/npdraw_bench.py > $O/bench.txt 2>&1
rc=$?; echo "bench rc=$rc"; cat $O/bench.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python tools/npdraw_bench.py 65536 64 > $O/prof.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --kernel-include-regex "np_" --output-format csv -d $O/pmc -o run -- python tools/npdraw_bench.py 65536 64 > $O/pmc.log 2>&1
rc=$?; echo "pmc rc=$rc"; exit $rc
