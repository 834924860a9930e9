set -u
cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out; export TMPDIR=/tmp
NS="2 4" WORKLOADS="caustic8 cornell1080" STEPS_N=4 bash scripts/rehearse.sh || exit 1
NS="2" WORKLOADS="weak64" STEPS_N=2 bash scripts/rehearse.sh || exit 1
for f in gpurun_out/rehearse_caustic8_2.log gpurun_out/rehearse_caustic8_4.log gpurun_out/rehearse_cornell1080_2.log gpurun_out/rehearse_cornell1080_4.log gpurun_out/rehearse_weak64_2.log; do
grep '^{' $f | tail -1 | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
sb=d['scaling_breakdown']
print('$f', d['n_gpus'], d['value'], d['reduce_backend'], 'render', sb['render_s'], 'reduce', sb['reduce_s'])"
done
