#!/bin/bash
# round 4 s25: pass tables in the kernel arguments, pool counters zeroed by the previous pooled
# launch: parity, caustic probe, bench cornell / caustic8
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_pool.py tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_multi.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s25_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/s25_pytest.log; [ $rc -eq 0 ] || exit $rc
echo "== caustic probe (auto)"
timeout -k 10 300 python scripts/shard_probe.py --scene caustic --passes 128 --strong --ns 1,2,4,8 --reps 10 > gpurun_out/s25_probe.log 2>&1 || exit 7
grep '^{' gpurun_out/s25_probe.log | grep '"streams_req": 0'
for sc in "--workload caustic8" "--scene cornell"; do
  echo "== $sc"
  VARIANTS="A:BDPT_POOL=" BENCH_ARGS="$sc --steps 10" ROUNDS=2 bash scripts/ab_env.sh || exit 5
done
