#!/bin/bash
# round 4 s31: restart group size (BDPT_REGEN_K) for the pass-stream kernel on cornell (auto mode)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
VARIANTS="K48:BDPT_JIT_FLAGS= K40:BDPT_JIT_FLAGS=-DBDPT_REGEN_K=40 K56:BDPT_JIT_FLAGS=-DBDPT_REGEN_K=56 K64:BDPT_JIT_FLAGS=-DBDPT_REGEN_K=64" \
  BENCH_ARGS="--scene cornell --steps 10" ROUNDS=2 bash scripts/ab_env.sh || exit 5
