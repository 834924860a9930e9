set -u
cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_specialize.py -q -k synthetic64 --timeout 200 --timeout-method thread > gpurun_out/spec64.log 2>&1 || { tail -20 gpurun_out/spec64.log; exit 1; }
tail -2 gpurun_out/spec64.log
for sp in 0 1 0 1; do timeout -k 10 300 python bench.py --workload weak64 --no-cpu-baseline --specialize $sp --steps 10 > gpurun_out/ab64_$sp.log 2>&1 || exit 1; python -c "import json;d=json.loads(open('gpurun_out/ab64_$sp.log').read().strip().splitlines()[-1]);print('spec',$sp,d['value'],d['config']['specialized'],d['config']['pass_streams'])"; done
