set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests -m gpu -q -rf -x > gpurun_out/t19.log 2>&1; rc=$?; tail -3 gpurun_out/t19.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python tools/stamps.py mppi_robotarm_amd/_lib/libmppi_rocm_stamps.so 65536 64 5 > gpurun_out/st19.log 2>&1 || exit $?
LAMBDA=3e6 timeout -k 10 200 python tools/stamps.py mppi_robotarm_amd/_lib/libmppi_rocm_stamps.so 65536 64 3 >> gpurun_out/st19.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > gpurun_out/b19.log 2>&1 || exit $?
cat gpurun_out/b19.log | tail -1
