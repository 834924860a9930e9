#!/bin/bash
# A/B bench of variant libraries (variants/<name>/libbdpt.so) against the default build, in one
# GPU session; ROUNDS interleaved rounds.  Usage: VARIANTS="a b" bash scripts/ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in default ${VARIANTS}; do
    if [ "$v" = default ]; then lib=""; else lib="variants/$v/libbdpt.so"; fi
    BDPT_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/ab_$v.log 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "STOP $v rc=$rc"; tail -5 gpurun_out/ab_$v.log; exit $rc; fi
    echo "round $r $v $(python -c "import json,sys; d=json.loads(open('gpurun_out/ab_$v.log').read().strip().splitlines()[-1]); print(d['value'], d['device_ms_per_step'])")"
  done
done
