#!/bin/bash
# GPU box: -m gpu suite, then the trajectory re-roll timed for the saved
# build (libmppi_rocm_base.so) and the product, arm and chain, and a rocprof
# kernel-trace summary of the product's arm re-roll.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/traj; mkdir -p $O
L=mppi_robotarm_amd/_lib
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rf > $O/gputest.log 2>&1
rc=$?; echo "gputest rc=$rc"; tail -3 $O/gputest.log; [ $rc -eq 0 ] || { tail -60 $O/gputest.log; exit $rc; }
for lib in libmppi_rocm_base.so libmppi_rocm.so; do
  timeout -k 10 120 python tools/traj_bench.py $L/$lib 2>/dev/null | sed "s/^/$lib arm: /" || exit 1
  WORKLOAD=c5 timeout -k 10 120 python tools/traj_bench.py $L/$lib 2>/dev/null | sed "s/^/$lib c5: /" || exit 1
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/traj_bench.py > $O/prof.log 2>&1 || exit 1
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs cat | cut -c1-160
