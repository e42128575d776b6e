#!/bin/bash
# Bench sweep over the BASELINE configs that fit one GPU (one line per config),
# plus a 2-rank rehearsal of the multi-GPU path on the one GPU (gloo: RCCL refuses two ranks on one GPU;
# the in-launch exchange needs the process group only for the IPC handles).  Logs under gpurun_out/sweep/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/sweep; mkdir -p $O
run() { local n=$1; shift; timeout -k 10 300 "$@" > $O/$n.log 2>&1; local rc=$?; echo "$n rc=$rc"; grep -h '^{' $O/$n.log | python3 -c "import sys,json; [print('   ', j['config']['workload'][:60], '| ms/step %.4f | value %.3e | kernel_ms %.4f' % (j['ms_per_step'], j['value'], j['kernel_ms'])) for j in map(json.loads, sys.stdin)]"; [ $rc -le 1 ] || exit $rc; }
sel() { [ -z "${ONLY:-}" ] || [[ " $ONLY " == *" $1 "* ]]; }
sel c2 && run c2 python3 bench.py --K 4096 --T 32 --cpu-seconds 0
sel c3 && run c3 python3 bench.py --cpu-seconds 0
sel c3_graph && run c3_graph python3 bench.py --launch graph --cpu-seconds 0
sel c5 && run c5 python3 bench.py --workload c5 --steps 300 --warmup 30 --cpu-seconds 0
sel c3_n2 && run c3_n2 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 500 --warmup 50 --backend gloo
sel c3_n2_hoststaged && run c3_n2_hoststaged python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29532 bench.py --gpus 2 --steps 500 --warmup 50 --exchange rccl --backend gloo
