#!/bin/bash
# A/B of run-time settings in one GPU session: each variant is a list of VAR=VALUE environment
# assignments (no spaces inside a value), variants separated by '|', "" = the default; e.g.
# specialised-kernel compile options (BDPT_JIT_FLAGS; each option set has its own JIT cache entry):
#   VARIANTS="|BDPT_JIT_FLAGS=-DBDPT_SPLIT_TAIL=0" SCENES="cornell caustic" ROUNDS=2 bash scripts/ab_flags.sh
# (BENCH_EXTRA=--streams,16 in a variant adds bench.py arguments for that variant only)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
export BDPT_JIT_CACHE=$(mktemp -d /tmp/bdpt-jit-ab.XXXXXX)
IFS='|' read -r -a VS <<< "${VARIANTS:-|BDPT_JIT_FLAGS=-DBDPT_SPLIT_TAIL=0}"
for r in $(seq 1 ${ROUNDS:-2}); do
  for sc in ${SCENES:-cornell}; do
    k=0
    for v in "${VS[@]}"; do
      k=$((k+1))
      extra=""                                    # a variant's BENCH_EXTRA=--opt,value: extra bench args
      for kv in $v; do case "$kv" in BENCH_EXTRA=*) extra="${kv#BENCH_EXTRA=}"; extra="${extra//,/ }";; esac; done
      env $v timeout -k 10 300 python bench.py --no-cpu-baseline --scene $sc ${BENCH_ARGS:-} $extra > gpurun_out/abf_$k.log 2>&1
      rc=$?
      if [ $rc -ne 0 ]; then echo "STOP [$v] $sc rc=$rc"; tail -5 gpurun_out/abf_$k.log; exit $rc; fi
      echo "round $r $sc [${v:-default}] $(python -c "import json; d=json.loads(open('gpurun_out/abf_$k.log').read().strip().splitlines()[-1]); r=d['roofline'] or {}; print(d['value'], d['device_ms_per_step'], d['config']['specialized'], 'S=%d' % d['config']['pass_streams'], 'k=%s' % r.get('avg_launch_ms'))")"
    done
  done
done
