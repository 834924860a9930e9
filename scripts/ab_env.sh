#!/bin/bash
# A/B of environment settings in one GPU session: ROUNDS interleaved rounds of bench.py per
# variant.  VARIANTS="name1:ENV=1;ENV2=0 name2:ENV=0" (";" separates assignments, so a value may
# hold commas: BDPT_JIT_FLAGS=-DA=0,-DB=0) BENCH_ARGS="--scene caustic" bash scripts/ab_env.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in ${VARIANTS}; do
    name=${v%%:*}; envs=${v#*:}
    env $(echo "$envs" | tr ';' ' ') timeout -k 10 300 python bench.py --no-cpu-baseline --tail-seconds 0 ${BENCH_ARGS:-} > gpurun_out/abe_$name.log 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "STOP $name rc=$rc"; tail -5 gpurun_out/abe_$name.log; exit $rc; fi
    echo "round $r $name $(python -c "import json; d=json.loads(open('gpurun_out/abe_$name.log').read().strip().splitlines()[-1]); print(d['value'], d['device_ms_per_step'], d['config']['pass_streams'], d['roofline']['kernel_features'] if d['roofline'] else '')")"
  done
done
