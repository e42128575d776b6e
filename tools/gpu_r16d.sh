#!/bin/bash
# round 6: config 5's shard, four against eight lanes per sample (tools/ubench_chain_lanes.hip, both broadcast
# forms), then the NumPy draw's stride sweep (tools/gpu_npdraw.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r16d; mkdir -p $O
for sw in 0 1; do
  for K in 16384 8192 32768; do
    timeout -k 10 60 tools/_build/ubench_chain_lanes_sw$sw $K 128 20 >> $O/chain_lanes.jsonl 2>> $O/chain_lanes.err
    rc=$?; [ $rc -eq 0 ] || { echo "ubench rc=$rc"; cat $O/chain_lanes.err; exit $rc; }
  done
done
cat $O/chain_lanes.jsonl
STRIDES="64 128 256 512 1024" bash tools/gpu_npdraw.sh r16np
