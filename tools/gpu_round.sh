#!/bin/bash
# One GPU-box session: each GPU step under its own timeout; stop at the first
# fault / abort / timeout (rc not in {0, 1}).  Logs go to gpurun_out/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for s in "$@"; do
  case $s in
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()";;
    test)  step test 900 python -m pytest tests -m gpu -q -rf;;
    bench) step bench 600 python bench.py --steps 200 --warmup 20 --cpu-seconds 10;;
    benchq) step benchq 300 python bench.py --steps 100 --warmup 10 --cpu-seconds 0;;
    lat) step lat 300 python tools/latency_breakdown.py;;
    prof)  step prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 100 --warmup 10 --cpu-seconds 0;;
    *) echo "unknown step $s"; exit 2;;
  esac
done
