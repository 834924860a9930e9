#!/bin/bash
# round 5 session 8: full GPU suite with the unit fold in the auto mode, then the bench lines
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "STOP $1 rc=$2"; exit $2; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s8_pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/s8_pytest_gpu.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && stop tests $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/s8_bench_cornell.log 2>&1 || stop bench $?
tail -1 gpurun_out/s8_bench_cornell.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('cornell1080', d['value'], d['ms_per_step'], d['config']['pass_streams'], d['roofline']['kernel_features'], d['scaling_breakdown']['per_device'][0]['mode'])"
timeout -k 10 300 python bench.py --workload caustic8 --no-cpu-baseline > gpurun_out/s8_bench_caustic8.log 2>&1 || stop caustic8 $?
tail -1 gpurun_out/s8_bench_caustic8.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('caustic8', d['value'], d['ms_per_step'], d['config']['pass_streams'], d['roofline']['kernel_features'], d['scaling_breakdown']['per_device'][0]['mode'])"
