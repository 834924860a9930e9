#!/bin/bash
# round 4 s36: pool chunks of 64 pixels in the last quarter of a part (T) vs full chunks (F)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_pool.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s36_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/s36_pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in "T:" "F:-DBDPT_POOL_TAIL=0"; do
    name=${v%%:*}; fl=${v#*:}
    BDPT_JIT_FLAGS=$fl timeout -k 10 300 python scripts/shard_probe.py --scene caustic --passes 128 --strong --ns 1,8 --reps 10 > gpurun_out/s36_$name.log 2>&1 || exit 7
    echo "round $r $name"; grep '^{' gpurun_out/s36_$name.log | grep '"streams_req": 0'
  done
done
