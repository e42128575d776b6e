#!/bin/bash
# Launch-call cost against kernel-argument size (tools/launch_cost.hip, built in-tree beforehand),
# standalone and inside a PyTorch process.
set -o pipefail
mkdir -p gpurun_out/launch
timeout -k 10 120 tools/_build/launch_cost > gpurun_out/launch/default.txt 2>&1 &&
timeout -k 10 180 python tools/launch_cost_torch.py > gpurun_out/launch/in_torch.txt 2>&1
rc=$?
cat gpurun_out/launch/default.txt gpurun_out/launch/in_torch.txt
exit $rc
