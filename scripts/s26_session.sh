#!/bin/bash
# round 4 s26: pixel pools (forced) with other restart group sizes (BDPT_REGEN_K) on cornell and caustic8
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for sc in "--scene cornell:16" "--workload caustic8:16"; do
  args=${sc%%:*}; R=${sc##*:}
  echo "== $args (pools forced, chunk $R)"
  VARIANTS="K48:BDPT_POOL=$R K32:BDPT_POOL=$R;BDPT_JIT_FLAGS=-DBDPT_REGEN_K=32 K16:BDPT_POOL=$R;BDPT_JIT_FLAGS=-DBDPT_REGEN_K=16 K56:BDPT_POOL=$R;BDPT_JIT_FLAGS=-DBDPT_REGEN_K=56" \
    BENCH_ARGS="$args --steps 8 --streams 128" ROUNDS=1 bash scripts/ab_env.sh || exit 5
done
