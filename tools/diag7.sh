set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -q -x > gpurun_out/t7.log 2>&1; rc=$?; tail -3 gpurun_out/t7.log; [ $rc -le 1 ] || exit $rc
MPPI_LIB_PATH=$PWD/mppi_robotarm_amd/_lib/libmppi_rocm_native.so timeout -k 10 300 python -m pytest tests -m gpu -q > gpurun_out/t7n.log 2>&1; rc=$?; tail -3 gpurun_out/t7n.log; [ $rc -le 1 ] || exit $rc
for B in 256 512; do
  MPPI_BLOCK=$B timeout -k 10 200 python tools/stamps.py mppi_robotarm_amd/_lib/libmppi_rocm_stamps.so 65536 64 5 > gpurun_out/st7_$B.log 2>&1 || exit $?
  MPPI_BLOCK=$B MPPI_LIB_PATH=$PWD/mppi_robotarm_amd/_lib/libmppi_rocm_native.so timeout -k 10 300 python bench.py --steps 200 --warmup 20 --cpu-seconds 0 > gpurun_out/b7_$B.log 2>&1 || exit $?
done
MPPI_BLOCK=512 timeout -k 10 200 python tools/stamps.py mppi_robotarm_amd/_lib/libmppi_rocm_stampsacc.so 65536 64 5 > gpurun_out/st7_acc.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --cpu-seconds 0 > gpurun_out/b7_prod.log 2>&1 || exit $?
