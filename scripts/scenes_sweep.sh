#!/bin/bash
# Every reference scene through bench.py (1921x1081, auto stream mode, --passes P, default 32 for
# comparison with the round-2 and earlier round-3 sweeps): one line per scene with Ms/s, the
# stream count and traversal the run settled on.  Output: gpurun_out/scenes.txt
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; : > gpurun_out/scenes.txt
export BDPT_JIT_CACHE=$(mktemp -d /tmp/bdpt-jit-sc.XXXXXX)
for f in assets/scenes/*.scn; do
  s=$(basename "$f" .scn)
  timeout -k 10 300 python bench.py --no-cpu-baseline --scene "$s" --passes "${PASSES:-32}" --steps "${STEPS:-10}" \
      > gpurun_out/scene_$s.log 2>&1 || { echo "STOP $s"; tail -5 gpurun_out/scene_$s.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/scene_$s.log').read().strip().splitlines()[-1]); c=d['config']
f = (d.get('roofline') or {}).get('kernel_features', [])
print('$s', round(d['value']), 'S=%d' % c['pass_streams'], c['traversal'], 'pools' if 'pixel_pools' in f else '')" >> gpurun_out/scenes.txt
done
cat gpurun_out/scenes.txt
