set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
L=gpurun_out/d20.log; : > $L
timeout -k 10 300 python tools/ab.py mppi_robotarm_amd/_lib/libmppi_rocm_A.so mppi_robotarm_amd/_lib/libmppi_rocm_C.so >> $L 2>&1 || exit $?
for args in "" "--no-graph" "--nbuf 8" "--nbuf 8 --no-graph" "--nbuf 2" "--nbuf 2 --no-graph"; do
  echo "== bench $args" >> $L
  timeout -k 10 200 python bench.py --steps 400 $args 2>&1 | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step']*1e3,2), 'us/step; kernel', round(d['kernel_ms']*1e3,2))" >> $L || exit $?
done
