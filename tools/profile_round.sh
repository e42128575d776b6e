#!/bin/bash
# Round profile: kernel-trace stats of the bench, PMC traffic passes (one counter
# set per pass, no trace domains) for the rollout kernel and the calibration
# kernel.  Outputs under gpurun_out/prof_<tag>/.   Usage: tools/profile_round.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r01}
O=gpurun_out/prof_$TAG; mkdir -p $O
WL=${2:-c3}
XA=${3:-}   # extra bench.py arguments, e.g. "--K 16384"
# stats pass: the bench as it runs (clock settle, 1000 timed steps); PMC passes:
# few launches, no settle (byte counts do not depend on the clock, and every
# PMC dispatch is serialised)
B="python3 bench.py --workload $WL $XA --steps 1000 --warmup 100 --cpu-seconds 0"
BP="python3 bench.py --workload $WL $XA --steps 40 --warmup 4 --settle-ms 0 --cpu-seconds 0"
if [ "$WL" = c5 ]; then KR=chain_rollout; CA=4; else KR=rollout; CA=8; fi
# the calibration kernel is a git-ignored build product: compile it on the box
[ -x tools/calib_fetch ] || hipcc --offload-arch=gfx950 -O3 tools/calib_fetch.hip -o tools/calib_fetch 2>/dev/null || exit 3
step() { local n=$1; shift; timeout -k 10 400 "$@" > $O/$n.log 2>&1; local rc=$?; echo "$n rc=$rc"; [ $rc -le 1 ] || exit $rc; }
step stats rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- $B
step fetch rocprofv3 --pmc FETCH_SIZE --kernel-include-regex $KR --output-format csv -d $O/fetch -o p -- $BP
step write rocprofv3 --pmc WRITE_SIZE --kernel-include-regex $KR --output-format csv -d $O/write -o p -- $BP
step cfetch rocprofv3 --pmc FETCH_SIZE --kernel-include-regex calib --output-format csv -d $O/cfetch -o p -- ./tools/calib_fetch $CA
step cwrite rocprofv3 --pmc WRITE_SIZE --kernel-include-regex calib --output-format csv -d $O/cwrite -o p -- ./tools/calib_fetch $CA
step sq rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES --kernel-include-regex $KR --output-format csv -d $O/sq -o p -- $BP
step grbm rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --kernel-include-regex $KR --output-format csv -d $O/grbm -o p -- $BP
