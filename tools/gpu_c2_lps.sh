set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/c2ab; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "lanes_per_sample or large_rollout" > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do for l in 4 8; do
timeout -k 10 200 python bench.py --workload c2 --lps $l --steps 2000 --warmup 100 --cpu-seconds 0 > $O/b_${l}_$r.json 2>/dev/null || exit 1
python -c "import json;d=json.load(open('$O/b_${l}_$r.json'));print('lps',$l,'ms',round(d['kernel_ms']*1e3,2),'lat',round(d['control_step_latency_ms']*1e3,1))"
done; done
