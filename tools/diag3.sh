set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for v in l0 l1; do
  MPPI_LIB_PATH=$PWD/mppi_robotarm_amd/_lib/libmppi_rocm_$v.so timeout -k 10 300 python bench.py --steps 200 --warmup 20 --cpu-seconds 0 > gpurun_out/b3_$v.log 2>&1 || exit $?
done
timeout -k 10 200 python tools/stamps.py mppi_robotarm_amd/_lib/libmppi_rocm_l0s.so 65536 64 6 > gpurun_out/st3_l0s.log 2>&1 || exit $?
bash tools/pmc.sh l0 || exit $?
bash tools/pmc.sh l1 || exit $?
