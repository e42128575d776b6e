#!/bin/bash
# GPU box: the noise-stream tests (device Philox vs oracle/philox_ref.py, achieved errors recorded),
# then the Philox draw A/B (library transcendentals + mul_lo/mul_hi vs hardware + v_mad_u64_u32) and
# the c3 bench line (drop-in latency, back to back).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/philox; mkdir -p $O
rm -f $O/records.jsonl
export MPPI_PARITY_RECORD=$PWD/$O/records.jsonl
timeout -k 10 300 python -u -m pytest tests/test_gpu_noise_stream.py tests/test_gpu_index_parity.py -v --timeout 240 --timeout-method thread -rf > $O/test.log 2>&1
rc=$?; grep -E "passed|failed" $O/test.log | tail -2; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/test.log | head -30; exit $rc; }
WORKLOAD=philox timeout -k 10 120 python tools/ab.py mppi_robotarm_amd/_lib/libmppi_rocm_phlib.so mppi_robotarm_amd/_lib/libmppi_rocm.so 65536 64 30 50 > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
cat $O/ab.log
timeout -k 10 300 python bench.py --workload c3 > $O/bench_c3.json 2> $O/bench_c3.err || { tail -30 $O/bench_c3.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_c3.json'));print('c3 kernel_us', round(d['kernel_ms']*1e3,2), 'lat_ms', d['control_step_latency_ms'], 'b2b', d.get('control_step_latency_back_to_back_ms'))"
