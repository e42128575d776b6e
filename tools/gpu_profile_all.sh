#!/bin/bash
# GPU box: the round's profiles for c3, c2 and c5 (tools/profile_round.sh each),
# then the three bench lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r09}
bash tools/profile_round.sh $TAG c3 || exit $?
bash tools/profile_round.sh ${TAG}c2 c2 || exit $?
bash tools/profile_round.sh ${TAG}c5 c5 || exit $?
mkdir -p gpurun_out/bench_$TAG
for W in c3 c2 c5; do
  timeout -k 10 400 python bench.py --workload $W > gpurun_out/bench_$TAG/$W.json 2> gpurun_out/bench_$TAG/$W.err || { tail -20 gpurun_out/bench_$TAG/$W.err; exit 1; }
done
echo done
