set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -m gpu -q -rf > gpurun_out/t12.log 2>&1; rc=$?; tail -3 gpurun_out/t12.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python tools/stamps.py mppi_robotarm_amd/_lib/libmppi_rocm_stamps.so 65536 64 5 > gpurun_out/st12.log 2>&1 || exit $?
LAMBDA=3e6 timeout -k 10 200 python tools/stamps.py mppi_robotarm_amd/_lib/libmppi_rocm_stamps.so 65536 64 3 >> gpurun_out/st12.log 2>&1 || exit $?
timeout -k 10 300 python -m mppi_robotarm_amd.harness --ticks 200 > gpurun_out/h12.log 2>&1 || exit $?
timeout -k 10 300 python -m mppi_robotarm_amd.harness --ticks 200 --noise device --no-sampled >> gpurun_out/h12.log 2>&1 || exit $?
timeout -k 10 300 python -m mppi_robotarm_amd.harness --ticks 100 --noise device --no-sampled --K 65536 --T 64 >> gpurun_out/h12.log 2>&1 || exit $?
