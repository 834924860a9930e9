set -u
cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_units.py tests/test_gpu_parity.py -k "units or auto_streams" -x -q --timeout 120 --timeout-method thread > gpurun_out/s10_pytest.log 2>&1 || { tail -20 gpurun_out/s10_pytest.log; exit 1; }
tail -2 gpurun_out/s10_pytest.log
NS="2 4" WORKLOADS="cornell1080" STEPS_N=4 bash scripts/rehearse.sh || exit 1
for n in 2 4; do grep '^{' gpurun_out/rehearse_cornell1080_$n.log | tail -1 > gpurun_out/s10_rehearse_$n.json; done
timeout -k 10 300 python bench.py --gpus 2 --devices 0,0 --steps 5 --no-cpu-baseline > gpurun_out/s10_inproc.log 2>&1 || { tail -20 gpurun_out/s10_inproc.log; exit 1; }
grep '^{' gpurun_out/s10_inproc.log | tail -1 > gpurun_out/s10_inproc.json
for f in gpurun_out/s10_rehearse_2.json gpurun_out/s10_rehearse_4.json gpurun_out/s10_inproc.json; do
python3 -c "
import json; d=json.load(open('$f'))
print('$f', d['n_gpus'], d['value'], d['reduce_backend'], 'fallback', d.get('reduce_fallback'), 'choice_from', d.get('stream_choice_from'))
for p in d['scaling_breakdown']['per_device']: print('   ', p.get('rank', p.get('device')), p['mode'])"
done
timeout -k 10 120 python scripts/probe_step.py --scene cornell --streams 64 --tag units8 > gpurun_out/s10_probe.txt 2>&1 && BDPT_UNITS=8 timeout -k 10 120 python scripts/probe_step.py --scene cornell --streams 64 --tag units8 >> gpurun_out/s10_probe.txt 2>&1; grep '^{' gpurun_out/s10_probe.txt | cut -c1-150
