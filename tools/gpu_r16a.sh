#!/bin/bash
# round 6, first GPU pass: the read-back tests and sampled legs, then the whole -m gpu suite on the build
# without the A/B variants.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r16a; mkdir -p $O
lscpu > $O/lscpu.txt 2>&1
bash tools/gpu_sampled.sh --quick || exit 1
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rf > $O/gputest.log 2>&1
rc=$?; echo "full gputest rc=$rc"; tail -3 $O/gputest.log; exit $rc
