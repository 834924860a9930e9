#!/bin/bash
# round 4 s32: cornell weak-scaling rehearsal with the final build (one rank's share on one GPU,
# N x 128 passes per step), and the in-process two-shard context on one GPU
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python scripts/shard_probe.py --scene cornell --passes 128 --ns 1,2,4,8 --reps 3 > gpurun_out/s32_probe.log 2>&1 || exit 7
grep '^{' gpurun_out/s32_probe.log
timeout -k 10 300 python bench.py --gpus 2 --devices 0,0 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/s32_inproc.log 2>&1 || exit 8
tail -1 gpurun_out/s32_inproc.log | cut -c1-300
