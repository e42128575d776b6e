set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 200 python tools/stamps.py mppi_robotarm_amd/_lib/libmppi_rocm_stamps.so 65536 64 12 > gpurun_out/st_acc.log 2>&1 || exit $?
timeout -k 10 200 python tools/stamps.py mppi_robotarm_amd/_lib/libmppi_rocm_stamps_native.so 65536 64 12 > gpurun_out/st_nat.log 2>&1 || exit $?
LPS=1 timeout -k 10 200 python tools/stamps.py mppi_robotarm_amd/_lib/libmppi_rocm_stamps_native.so 65536 64 6 > gpurun_out/st_nat1.log 2>&1 || exit $?
LPS=4 timeout -k 10 200 python tools/stamps.py mppi_robotarm_amd/_lib/libmppi_rocm_stamps_native.so 65536 64 6 > gpurun_out/st_nat4.log 2>&1 || exit $?
