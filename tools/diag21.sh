set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests -m gpu -q -rf -x > gpurun_out/t21.log 2>&1; rc=$?; tail -2 gpurun_out/t21.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/b21.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --launch graph --cpu-seconds 0 > gpurun_out/b21g.log 2>&1 || exit $?
bash tools/profile_round.sh r02 || exit $?
