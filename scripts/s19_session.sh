#!/bin/bash
# round 4 s19: pixel pools with one queue over the launch's passes: chunk / grid / passes sweep
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for RGP in "16 64 128" "64 64 32" "64 256 32" "32 128 64"; do
  set -- $RGP
  echo "== pools chunk $1 grid $2 passes $3"
  BDPT_POOL=$1 BDPT_POOL_GRID=$2 BDPT_POOL_PASSES=$3 timeout -k 10 300 python scripts/shard_probe.py --scene caustic --passes 128 --strong --ns 1,8 --reps 10 --streams 128 > gpurun_out/s19_probe_$1_$2_$3.log 2>&1 || exit 8
  grep '^{' gpurun_out/s19_probe_$1_$2_$3.log | grep '"streams_req": 128'
done
