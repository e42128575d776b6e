set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for K in 8192 16384 32768 65536 131072 262144; do
  LPS=2 timeout -k 10 200 python tools/stamps.py mppi_robotarm_amd/_lib/libmppi_rocm_none.so $K 64 3 > gpurun_out/st5_none_$K.log 2>&1 || exit $?
done
for K in 65536 131072; do
  LPS=1 timeout -k 10 200 python tools/stamps.py mppi_robotarm_amd/_lib/libmppi_rocm_none.so $K 64 3 > gpurun_out/st5_none1_$K.log 2>&1 || exit $?
done
timeout -k 10 200 python tools/stamps.py mppi_robotarm_amd/_lib/libmppi_rocm_base.so 65536 64 3 > gpurun_out/st5_base.log 2>&1 || exit $?
