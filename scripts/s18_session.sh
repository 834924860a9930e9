#!/bin/bash
# round 4 s18: pixel pools with chunks claimed from per-pass counters: parity, then the caustic
# probe (N = 1, 8) over chunk and grid sizes, and the bench on caustic8 / cornell
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_pool.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s18_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/s18_pytest.log; [ $rc -eq 0 ] || exit $rc
for RG in "4 16" "4 64" "8 64" "16 64"; do
  set -- $RG
  echo "== pools chunk $1 grid $2"
  BDPT_POOL=$1 BDPT_POOL_GRID=$2 timeout -k 10 300 python scripts/shard_probe.py --scene caustic --passes 128 --strong --ns 1,8 --reps 10 --streams 128 > gpurun_out/s18_probe_$1_$2.log 2>&1 || exit 8
  grep '^{' gpurun_out/s18_probe_$1_$2.log | grep '"streams_req": 128'
done
