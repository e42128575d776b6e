set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rf > gpurun_out/gputest.log 2>&1
rc=$?; echo "gputest rc=$rc"; tail -3 gpurun_out/gputest.log; [ $rc -eq 0 ] || { tail -60 gpurun_out/gputest.log; exit $rc; }
timeout -k 10 300 python tools/latency_breakdown.py > gpurun_out/lat.log 2>&1; cat gpurun_out/lat.log
