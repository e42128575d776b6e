#!/bin/bash
# round 6: the device NumPy draw with a general 2 x 2 Sigma — draw tests, host RNG tests, latency legs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r16b; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_npdraw.py tests/test_gpu_multigpu_dropin.py -x -v --timeout 300 --timeout-method thread > $O/npdraw.log 2>&1
rc=$?; echo "npdraw rc=$rc"; grep -E "passed|failed" $O/npdraw.log | tail -2; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/npdraw.log | head -30; exit $rc; }
timeout -k 10 300 python -u -c "
import bench, json, numpy as np
r = {}
r['diag'] = bench.numpy_noise_latency(65536, 64, 0)
r['general'] = bench.numpy_noise_latency(65536, 64, 0, sigma=np.array([[20.0, 6.0], [6.0, 12.0]]))
print(json.dumps(r))
" > $O/lat.json 2> $O/lat.err || { tail $O/lat.err; exit 1; }
cat $O/lat.json
