#!/bin/bash
# Round 3 profiles: rocprofv3 kernel stats + separate PMC passes for c3, c2, c5 and config 5's 8-way shard
# (K = 16384 per GPU), then the bench lines (c3 with its CPU baseline).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/profile_round.sh r11 c3 || exit $?
bash tools/profile_round.sh r11c2 c2 || exit $?
bash tools/profile_round.sh r11c5 c5 || exit $?
bash tools/profile_round.sh r11c5k16384 c5 "--K 16384" || exit $?
O=gpurun_out/bench_r11; mkdir -p $O
timeout -k 10 400 python bench.py > $O/c3.json 2> $O/c3.err || { tail -20 $O/c3.err; exit 1; }
for W in c2 c5; do
  timeout -k 10 400 python bench.py --workload $W > $O/$W.json 2> $O/$W.err || { tail -20 $O/$W.err; exit 1; }
done
timeout -k 10 400 python bench.py --workload c5 --K 16384 --cpu-seconds 0 > $O/c5_k16384.json 2> $O/c5_k16384.err || exit 1
timeout -k 10 400 python bench.py --workload c5 --precision f64 --cpu-seconds 0 > $O/c5_f64.json 2> $O/c5_f64.err || exit 1
echo done
