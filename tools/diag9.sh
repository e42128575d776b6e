set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -m gpu -q -rf > gpurun_out/t9.log 2>&1; rc=$?; tail -5 gpurun_out/t9.log; [ $rc -le 1 ] || exit $rc
for L in 1 2 4; do LPS=$L timeout -k 10 200 python tools/stamps.py mppi_robotarm_amd/_lib/libmppi_rocm_stamps.so 65536 64 3 >> gpurun_out/st9.log 2>&1 || exit $?; done
LAMBDA=3e6 timeout -k 10 200 python tools/stamps.py mppi_robotarm_amd/_lib/libmppi_rocm_stamps.so 65536 64 3 >> gpurun_out/st9.log 2>&1 || exit $?
for K in 16384 32768 131072 262144; do for L in 1 2; do LPS=$L timeout -k 10 200 python tools/stamps.py mppi_robotarm_amd/_lib/libmppi_rocm_stamps.so $K 64 3 >> gpurun_out/st9.log 2>&1 || exit $?; done; done
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --cpu-seconds 0 > gpurun_out/b9.log 2>&1 || exit $?
