set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r07
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r07/test.log 2>&1 || { echo test rc=$?; tail -30 gpurun_out/r07/test.log; exit 1; }
tail -2 gpurun_out/r07/test.log
timeout -k 10 300 python tools/latency_breakdown.py > gpurun_out/r07/lat.log 2>&1 || { echo lat rc=$?; tail gpurun_out/r07/lat.log; exit 1; }
cat gpurun_out/r07/lat.log
timeout -k 10 300 python bench.py --steps 300 --warmup 30 --cpu-seconds 0 > gpurun_out/r07/bench.log 2>&1 || exit 1
grep -o '"control_step_latency_ms": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/r07/bench.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r07/stats -o run -- python3 bench.py --steps 300 --warmup 30 --cpu-seconds 0 > gpurun_out/r07/prof.log 2>&1 || exit 1
find gpurun_out/r07/stats -name '*kernel_stats.csv' | xargs cut -c1-60,150-260
