set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for v in base nonoise noua nolookup none; do
  timeout -k 10 200 python tools/stamps.py mppi_robotarm_amd/_lib/libmppi_rocm_$v.so 65536 64 5 > gpurun_out/st4_$v.log 2>&1 || exit $?
done
