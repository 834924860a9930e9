#!/bin/bash
# The round-end driver sequence on the GPU box, from the tree as it travels (built here first with
# `python -c "import __graft_entry__ as e; e.build()"`): pytest -m gpu, smoke(), bench.py --gpus 1,
# then a rocprofv3 kernel-trace --stats run of the same bench command.  Each GPU step has its own
# time limit and the script stops at the first failure.  Outputs under gpurun_out/final_*.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
stop() { echo "STOP $1 (exit $2)"; exit "$2"; }
timeout -k 10 1200 python -u -m pytest tests -x -q -m gpu --timeout 600 --timeout-method thread --durations=12 \
    > gpurun_out/final_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/final_pytest_gpu.log; stop pytest $?; }
tail -16 gpurun_out/final_pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as e; e.smoke()" > gpurun_out/final_smoke.log 2>&1 || stop smoke $?
tail -1 gpurun_out/final_smoke.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/final_bench.log 2>&1 || stop bench $?
tail -1 gpurun_out/final_bench.log | cut -c1-300
rm -rf gpurun_out/final_prof
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/final_prof -o run --output-format csv -- \
    python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/final_prof.log 2>&1 || stop prof $?
grep path_kernel gpurun_out/final_prof/run_kernel_stats.csv | cut -c1-200
echo REHEARSAL_DONE
