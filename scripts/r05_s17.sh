set -u
cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s17_pytest.log 2>&1 || { tail -30 gpurun_out/s17_pytest.log; exit 1; }
tail -2 gpurun_out/s17_pytest.log
timeout -k 10 300 python bench.py --workload caustic8 > gpurun_out/s17_bench_caustic8.json 2> gpurun_out/s17_bench_caustic8.err || exit 1
tail -1 gpurun_out/s17_bench_caustic8.json | cut -c1-400
timeout -k 10 400 python bench.py > gpurun_out/s17_bench.json 2> gpurun_out/s17_bench.err || exit 1
tail -1 gpurun_out/s17_bench.json | cut -c1-400
