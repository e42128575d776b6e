set -u
cd "${GRAFT_REPO_ROOT:-.}"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "lanes_per_sample or large_rollout" --timeout 120 --timeout-method thread -rf > gpurun_out/lps16_tests.log 2>&1 || { tail -30 gpurun_out/lps16_tests.log; exit 1; }
tail -1 gpurun_out/lps16_tests.log
L=mppi_robotarm_amd/_lib/libmppi_rocm.so
for KT in "2048 32" "4096 32" "4096 64" "8192 32"; do
  LPS_LIST=4,8,16 timeout -k 10 120 python tools/ab.py $L $L $L $KT 2>/dev/null | grep -h "median\|K=" || exit 1
done
