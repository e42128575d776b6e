#!/bin/bash
# GPU box: the VALU issue-rate microbenchmark (profiles/ubench_issue.json) and the round's c3 / c2 profiles
# (tools/profile_round.sh: kernel-trace stats + separate PMC passes).  Usage: bash tools/gpu_roofline.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r15}
mkdir -p gpurun_out/ubench_$TAG
[ -x tools/ubench_issue ] || hipcc --offload-arch=gfx950 -O3 tools/ubench_issue.hip -o tools/ubench_issue 2>/dev/null || exit 3
timeout -k 10 120 ./tools/ubench_issue > gpurun_out/ubench_$TAG/ubench_issue.json || exit $?
bash tools/profile_round.sh $TAG c3 || exit $?
bash tools/profile_round.sh ${TAG}c2 c2 || exit $?
echo done
