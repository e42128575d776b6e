set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -q -x > gpurun_out/t2.log 2>&1; rc=$?; tail -3 gpurun_out/t2.log; [ $rc -le 1 ] || exit $rc
MPPI_LIB_PATH=$PWD/mppi_robotarm_amd/_lib/libmppi_rocm_native.so timeout -k 10 300 python -m pytest tests -m gpu -q > gpurun_out/t2n.log 2>&1; rc=$?; tail -3 gpurun_out/t2n.log; [ $rc -le 1 ] || exit $rc
for v in stamps stamps_native; do
  timeout -k 10 200 python tools/stamps.py mppi_robotarm_amd/_lib/libmppi_rocm_$v.so 65536 64 8 > gpurun_out/st2_$v.log 2>&1 || exit $?
  LPS=1 timeout -k 10 200 python tools/stamps.py mppi_robotarm_amd/_lib/libmppi_rocm_$v.so 65536 64 4 >> gpurun_out/st2_$v.log 2>&1 || exit $?
  LPS=4 timeout -k 10 200 python tools/stamps.py mppi_robotarm_amd/_lib/libmppi_rocm_$v.so 65536 64 4 >> gpurun_out/st2_$v.log 2>&1 || exit $?
done
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --cpu-seconds 0 > gpurun_out/b2.log 2>&1 || exit $?
MPPI_LIB_PATH=$PWD/mppi_robotarm_amd/_lib/libmppi_rocm_native.so timeout -k 10 300 python bench.py --steps 200 --warmup 20 --cpu-seconds 0 > gpurun_out/b2n.log 2>&1 || exit $?
