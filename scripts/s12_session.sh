set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused_variants.py tests/test_gpu_specialize.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s12_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/s12_pytest.log; [ $rc -eq 0 ] || exit $rc
V="A:BDPT_JIT_FLAGS= P:BDPT_JIT_FLAGS=-DBDPT_PAIR_AT_USE=0 B:BDPT_JIT_FLAGS=-DBDPT_RNG_BUF=0 O:BDPT_JIT_FLAGS=-DBDPT_RNG_BUF=0,-DBDPT_PAIR_AT_USE=0"
for sc in caustic open simple; do
  echo "== $sc"; VARIANTS="$V" BENCH_ARGS="--scene $sc --steps 10 --streams 1" ROUNDS=2 bash scripts/ab_env.sh || exit 5
done
echo "== caustic8"; VARIANTS="$V" BENCH_ARGS="--workload caustic8 --steps 10" ROUNDS=2 bash scripts/ab_env.sh
