#!/bin/bash
# round 4 s14: pixel pools on the open scenes: caustic8 (auto: fused vs pools), synthetic64, and
# the caustic strong-scaling probe with pools
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
echo "== caustic8"
VARIANTS="A:BDPT_POOL= P4:BDPT_POOL=4 P16:BDPT_POOL=16" BENCH_ARGS="--workload caustic8 --steps 10" ROUNDS=2 bash scripts/ab_env.sh || exit 5
echo "== synthetic64"
VARIANTS="A:BDPT_POOL= P4:BDPT_POOL=4" BENCH_ARGS="--scene synthetic64 --steps 10" ROUNDS=2 bash scripts/ab_env.sh || exit 6
echo "== caustic strong probe, pools 4"
BDPT_POOL=4 timeout -k 10 300 python scripts/shard_probe.py --scene caustic --passes 128 --strong --streams 1,128 > gpurun_out/s14_probe_p4.log 2>&1 || exit 7
cat gpurun_out/s14_probe_p4.log
