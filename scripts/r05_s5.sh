#!/bin/bash
# round 5 session 5: ordered in-kernel fold (BDPT_UNITS) -- parity first, then timing
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "STOP $1 rc=$2"; exit $2; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_units.py -x -q --timeout 120 --timeout-method thread > gpurun_out/s5_pytest_units.log 2>&1 || { tail -30 gpurun_out/s5_pytest_units.log; stop tests $?; }
tail -3 gpurun_out/s5_pytest_units.log
P=scripts/probe_step.py
O=gpurun_out/s5_units.txt
run() { tag=$1; shift; env "$@" timeout -k 10 150 python $P $ARGS --tag $tag >> $O 2>&1 || stop $tag $?; }
for r in 1 2; do
  ARGS="--scene cornell --streams 64"
  run k_s64 X=0
  run k_u2 BDPT_UNITS=2
  run k_u4 BDPT_UNITS=4
  run k_u8 BDPT_UNITS=8
  run k_u16 BDPT_UNITS=16
  run k_u32 BDPT_UNITS=32
  ARGS="--scene caustic --streams 128"
  run c_pools BDPT_POOL=16
  run c_u4 BDPT_UNITS=4
  run c_u16 BDPT_UNITS=16
  run c_u64 BDPT_UNITS=64
done
grep -v amdgpu.ids $O | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['tag'], d['streams'], d['ms_per_step'], d['kernel_ms'], d['Msamples_s'])"
