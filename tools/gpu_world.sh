#!/bin/bash
# One GPU call: the world 2/4/8 exchange rehearsal on one GPU (tests/test_gpu_exchange_world.py), the GPU suite,
# a bench.py --gpus 8 rehearsal line (8 ranks of K = 1536 on one GPU, in-launch exchange) and the N = 1 c3 line.
# Usage (on the box): bash tools/gpu_world.sh <outdir>
out=${1:-gpurun_out/world}
mkdir -p "$out"
fatal() { case $1 in 124|137|134|139) echo "fatal rc $1 in $2: stopping"; exit "$1";; esac; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_exchange_world.py -v --timeout 120 --timeout-method thread \
    > "$out/world.log" 2>&1
rc=$?; echo "world tests rc=$rc"; fatal $rc world
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread \
    --ignore=tests/test_gpu_exchange_world.py > "$out/gpu.log" 2>&1
rc=$?; echo "gpu suite rc=$rc"; tail -3 "$out/gpu.log"; fatal $rc suite
GPU_MAX_HW_QUEUES=1 timeout -k 10 300 python bench.py --gpus 8 --K 1536 --lps 1 --steps 500 --warmup 20 \
    --cpu-seconds 0 > "$out/bench_w8_k1536.json" 2> "$out/bench_w8_k1536.err"
rc=$?; echo "bench w8 rc=$rc"; fatal $rc bench_w8
GPU_MAX_HW_QUEUES=1 timeout -k 10 300 python bench.py --gpus 4 --K 1536 --lps 1 --steps 500 --warmup 20 \
    --cpu-seconds 0 > "$out/bench_w4_k1536.json" 2> "$out/bench_w4_k1536.err"
rc=$?; echo "bench w4 rc=$rc"; fatal $rc bench_w4
timeout -k 10 300 python bench.py --steps 1000 --warmup 100 --cpu-seconds 0 > "$out/bench_c3.json" 2> "$out/bench_c3.err"
rc=$?; echo "bench c3 rc=$rc"; fatal $rc bench_c3
exit 0
