#!/bin/bash
# The round-6 GPU sessions whose results are under profiles/r06_s<N>_* (one function per
# session; each ran as `gpurun -- bash scripts/r06_sessions.sh s<N>`).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp

pytest_gpu() {   # $1 = log name, rest = pytest selection
  local log=gpurun_out/$1; shift
  timeout -k 10 900 python -u -m pytest "$@" -m gpu -x -q --timeout 300 --timeout-method thread > "$log" 2>&1 \
    || { tail -30 "$log"; return 1; }
  tail -2 "$log"
}

s1() {
  # sin/cos planes (BDPT_SCP): the GPU suite, then bench A/B against the per-vertex fp64 sincos
  pytest_gpu s1_pytest_gpu.log tests || exit 1
  for w in cornell1080 caustic8 weak64; do
    MODE=bench ARGS="--workload $w --no-cpu-baseline" ROUNDS=2 \
      VARIANTS="scp: noscp:BDPT_JIT_FLAGS=-DBDPT_SCP=0" OUT=gpurun_out/s1_ab_scp.txt bash scripts/ab.sh || exit 1
  done
}

s2() {
  # the multi-device tests alone first (s1 aborted in bdpt_create_multi), then the rest as s1
  timeout -k 10 300 python -u -m pytest tests/test_gpu_multi.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/s2_multi.log 2>&1 || { grep -v "^  File" gpurun_out/s2_multi.log | tail -30; exit 1; }
  tail -2 gpurun_out/s2_multi.log
  pytest_gpu s2_pytest_gpu.log tests || exit 1
  for w in cornell1080 caustic8 weak64; do
    MODE=bench ARGS="--workload $w --no-cpu-baseline" ROUNDS=2 \
      VARIANTS="scp: noscp:BDPT_JIT_FLAGS=-DBDPT_SCP=0" OUT=gpurun_out/s2_ab_scp.txt bash scripts/ab.sh || exit 1
  done
}

"$@"
