set -u
cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "pool or auto or stream or fold or caustic or shard or config" > gpurun_out/s23_pytest.log 2>&1 || { tail -30 gpurun_out/s23_pytest.log; exit 1; }
tail -1 gpurun_out/s23_pytest.log
MODE=bench ARGS="--workload caustic8 --no-cpu-baseline --steps 20" ROUNDS=3 VARIANTS="bits:" OUT=gpurun_out/s23_ab.txt bash scripts/ab.sh || exit 1
rm -rf gpurun_out/prof_s23 && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_s23 -o run --output-format csv -- python3 bench.py --workload caustic8 --no-cpu-baseline --steps 10 > gpurun_out/prof_s23.log 2>&1 || exit 1
head -4 gpurun_out/prof_s23/run_kernel_stats.csv | cut -c1-150
