#!/bin/bash
# round 5 session 9: per-workload rocprof stats + PMC records (units for cornell1080), weak64 bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
WORKLOADS="cornell1080:64:cornell1080:BDPT_UNITS=8 caustic8:128:caustic8:BDPT_POOL=16 weak64:32" bash scripts/profile_workloads.sh
