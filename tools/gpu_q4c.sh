set -u
bash tools/gpu_ab.sh q4c "tests/test_gpu_chain.py" "WORKLOAD=c5 : libmppi_rocm_old.so libmppi_rocm.so 16384 128 16 20" || exit 1
O=gpurun_out/q4c
WARM=10 WORKLOAD=c5 timeout -k 10 120 python tools/stamps.py mppi_robotarm_amd/_lib/libmppi_rocm_stamp.so 16384 128 4 > $O/stamps_c5k16384.log 2>&1 || { tail $O/stamps_c5k16384.log; exit 1; }
tail -8 $O/stamps_c5k16384.log
