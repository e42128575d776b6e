set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -q > gpurun_out/t10.log 2>&1; rc=$?; tail -2 gpurun_out/t10.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --cpu-seconds 10 > gpurun_out/b10.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --cpu-seconds 0 --no-graph > gpurun_out/b10e.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke10.log 2>&1 || exit $?
