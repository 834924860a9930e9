#!/bin/bash
# round 4 s33: waves/SIMD target of the pass-stream build (pools on open scenes)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for sc in "--workload caustic8" "--scene open"; do
  echo "== $sc"
  VARIANTS="W6:BDPT_JIT_WAVES= W5:BDPT_JIT_WAVES=5" BENCH_ARGS="$sc --steps 10" ROUNDS=2 bash scripts/ab_env.sh || exit 5
done
