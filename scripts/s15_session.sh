#!/bin/bash
# round 4 s15: pool size sweep on the open scenes (bench, auto mode) and the caustic N = 8 probe
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
echo "== caustic8"
VARIANTS="A:BDPT_POOL= P16:BDPT_POOL=16 P32:BDPT_POOL=32 P64:BDPT_POOL=64" BENCH_ARGS="--workload caustic8 --steps 10" ROUNDS=2 bash scripts/ab_env.sh || exit 5
for sc in open simple; do
  echo "== $sc"
  VARIANTS="A:BDPT_POOL= P16:BDPT_POOL=16 P32:BDPT_POOL=32" BENCH_ARGS="--scene $sc --steps 10" ROUNDS=1 bash scripts/ab_env.sh || exit 6
done
for R in 16 32; do
  echo "== caustic strong probe, pools $R"
  BDPT_POOL=$R timeout -k 10 300 python scripts/shard_probe.py --scene caustic --passes 128 --strong --ns 1,8 --streams 128 > gpurun_out/s15_probe_p$R.log 2>&1 || exit 7
  grep '^{' gpurun_out/s15_probe_p$R.log
done
