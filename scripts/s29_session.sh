#!/bin/bash
# round 4 s29: same-box A/B of this tree (A) against the round-3 tree (R, ab_r03/: its own
# bench.py, package and library) on closed scenes at 128- and 32-pass steps
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
run() {  # $1 = name, $2 = dir, rest = bench args
  local name=$1 dir=$2; shift 2
  (cd $dir && timeout -k 10 300 python bench.py --no-cpu-baseline "$@") > gpurun_out/s29_$name.log 2>&1 || { echo "STOP $name"; tail -5 gpurun_out/s29_$name.log; exit 5; }
  python -c "import json; d=json.loads(open('gpurun_out/s29_$name.log').read().strip().splitlines()[-1]); print('$name', d['value'], d['device_ms_per_step'], d['config']['pass_streams'], d['devices'][0]['sclk']['current'])"
}
for r in 1 2; do
  for args in "--scene cornell --steps 10" "--scene cornell --passes 32 --steps 10" "--scene cornell_glass --passes 32 --steps 10"; do
    echo "== round $r: $args"
    run A . $args --tail-seconds 0
    run R ab_r03 $args
  done
done
