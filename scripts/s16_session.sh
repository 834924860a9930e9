#!/bin/bash
# round 4 s16: caustic strong-scaling probe (wall time per call, as the bench), pools against the
# current modes, N = 1 and 8
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
echo "== no pools (auto, fused, S = 32, S = 128)"
timeout -k 10 300 python scripts/shard_probe.py --scene caustic --passes 128 --strong --ns 1,8 --reps 10 --streams 1,32,128 > gpurun_out/s16_probe_p0.log 2>&1 || exit 7
grep '^{' gpurun_out/s16_probe_p0.log
for R in 8 16 32; do
  echo "== pools $R"
  BDPT_POOL=$R timeout -k 10 300 python scripts/shard_probe.py --scene caustic --passes 128 --strong --ns 1,8 --reps 10 --streams 128 > gpurun_out/s16_probe_p$R.log 2>&1 || exit 8
  grep '^{' gpurun_out/s16_probe_p$R.log
done
