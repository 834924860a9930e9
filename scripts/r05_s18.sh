set -u
cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "pool or auto or stream or fold or caustic or shard or config" > gpurun_out/s18_pytest.log 2>&1 || { tail -30 gpurun_out/s18_pytest.log; exit 1; }
tail -2 gpurun_out/s18_pytest.log
MODE=bench ARGS="--workload caustic8 --no-cpu-baseline --steps 20" ROUNDS=3 VARIANTS="sparse:" OUT=gpurun_out/s18_ab.txt bash scripts/ab.sh || exit 1
timeout -k 10 500 python scripts/shard_probe.py --scene caustic --passes 128 --strong --reps 20 --ns 1,8 > gpurun_out/s18_caustic_strong.txt 2>&1 || { tail -20 gpurun_out/s18_caustic_strong.txt; exit 1; }
tail -4 gpurun_out/s18_caustic_strong.txt
