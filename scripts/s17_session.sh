#!/bin/bash
# round 4 s17: kernel trace of the caustic N = 8 share (auto streams): path kernels, folds, gaps
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/s17_trace -o s17 --output-format csv -- python scripts/shard_probe.py --scene caustic --passes 128 --strong --ns 8 --reps 10 > gpurun_out/s17_probe.log 2>&1 || exit 7
grep '^{' gpurun_out/s17_probe.log
find gpurun_out/s17_trace -name "*.csv" | head
