#!/bin/bash
# GPU test pass on the box: the whole -m gpu suite (one process), verbose, per-test
# timeout; then the listed extra steps of tools/gpu_round.sh.  Logs in gpurun_out/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread -rf \
  ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/gputest.log 2>&1
rc=$?
echo "gputest rc=$rc"; grep -E "passed|failed|error" gpurun_out/gputest.log | tail -3
[ $rc -eq 0 ] || { tail -40 gpurun_out/gputest.log; exit $rc; }
[ $# -gt 0 ] && exec bash tools/gpu_round.sh "$@"
exit 0
