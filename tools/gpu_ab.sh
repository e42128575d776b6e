#!/bin/bash
# GPU box: a test selection, then one-process A/B timings (tools/ab.py) of library variants
# built with tools/build_variants.sh.  Usage: gpu_ab.sh OUT "pytest args" "ab spec" ["ab spec" ...]
#   ab spec: "ENV=.. ENV2=.. : lib1 lib2 ... [K T batches per]"  (libs relative to mppi_robotarm_amd/_lib)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/$1; shift; mkdir -p $O
export MPPI_PARITY_RECORD=$PWD/$O/parity_records.jsonl
if [ -n "$1" ]; then
  timeout -k 10 900 python -u -m pytest $1 -v --timeout 300 --timeout-method thread -rf -s > $O/tests.log 2>&1
  rc=$?; echo "tests rc=$rc"; grep -E "passed|failed" $O/tests.log | tail -2
  [ $rc -eq 0 ] || { grep -E "^FAILED|^E " $O/tests.log | head -30; exit $rc; }
fi
shift
i=0
for spec in "$@"; do
  envs=${spec%%:*}; args=${spec#*:}
  libs=""; nums=""
  for a in $args; do case $a in *.so) libs="$libs mppi_robotarm_amd/_lib/$a";; *) nums="$nums $a";; esac; done
  i=$((i+1))
  env $envs timeout -k 10 300 python -u tools/ab.py $libs $nums > $O/ab_$i.txt 2>&1 || { tail -20 $O/ab_$i.txt; exit 1; }
  echo "== ab $i: $envs"; cat $O/ab_$i.txt
done
