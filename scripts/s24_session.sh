#!/bin/bash
# round 4 s24: pool launch shape with interleaved passes: N = 8 share and whole frame
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for GR in "16 4" "32 4" "32 8" "64 8" "64 16"; do
  set -- $GR
  echo "== N=8 grid $1 chunk $2"
  BDPT_POOL=$2 BDPT_POOL_GRID=$1 timeout -k 10 300 python scripts/shard_probe.py --scene caustic --passes 128 --strong --ns 8 --reps 10 --streams 128 > gpurun_out/s24_8_$1_$2.log 2>&1 || exit 8
  grep '^{' gpurun_out/s24_8_$1_$2.log | grep '"streams_req": 128'
done
for GR in "32 8" "64 16" "128 16" "128 32"; do
  set -- $GR
  echo "== N=1 grid $1 chunk $2"
  BDPT_POOL=$2 BDPT_POOL_GRID=$1 timeout -k 10 300 python scripts/shard_probe.py --scene caustic --passes 128 --strong --ns 1 --reps 10 --streams 128 > gpurun_out/s24_1_$1_$2.log 2>&1 || exit 8
  grep '^{' gpurun_out/s24_1_$1_$2.log | grep '"streams_req": 128'
done
