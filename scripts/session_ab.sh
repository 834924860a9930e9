#!/bin/bash
# GPU session: selected parity tests, then an A/B of BDPT_JIT_FLAGS variants on several scenes.
#   TESTS="tests/test_gpu_specialize.py ..." FLAGS_B="-DBDPT_X=0" SCENES_AB="cornell caustic" bash scripts/session_ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/sab_pytest.log 2>&1
  rc=$?; tail -3 gpurun_out/sab_pytest.log; [ $rc -eq 0 ] || exit $rc
fi
for sc in ${SCENES_AB:-cornell}; do
  echo "== $sc"; VARIANTS="A:BDPT_JIT_FLAGS= B:BDPT_JIT_FLAGS=${FLAGS_B}" BENCH_ARGS="--scene $sc --steps ${STEPS_AB:-10} ${EXTRA_AB:-}" ROUNDS=${ROUNDS:-2} bash scripts/ab_env.sh || exit 5
done
