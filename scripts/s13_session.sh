#!/bin/bash
# round 4 s13: pass-stream kernel random loads (planar prefetch restored, settled q, park-time
# load) and pixel pools (BDPT_POOL), parity first
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_pool.py tests/test_gpu_specialize.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s13_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/s13_pytest.log; [ $rc -eq 0 ] || exit $rc
for sc in cornell cornell_glass; do
  echo "== $sc"
  VARIANTS="A:BDPT_JIT_FLAGS= O:BDPT_JIT_FLAGS=-DBDPT_PARK_LOAD=0,-DBDPT_Q_SETTLED=0,-DBDPT_PAIR_AT_USE=0 P2:BDPT_POOL=2 P4:BDPT_POOL=4 P8:BDPT_POOL=8" \
    BENCH_ARGS="--scene $sc --steps 10" ROUNDS=2 bash scripts/ab_env.sh || exit 5
done
