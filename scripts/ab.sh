#!/bin/bash
# The A/B driver for one GPU session: interleaved rounds of variants, each variant a set of
# environment assignments (kernel builds through BDPT_JIT_FLAGS / BDPT_LIB, modes through
# BDPT_UNITS / BDPT_POOL / ..., or nothing = the default), timed by scripts/probe_step.py (wall ms
# per step of back-to-back calls; ablations allowed) or by bench.py (MODE=bench: the metric line,
# frame checked).  One line per (round, variant): tag, streams, ms/step, path-kernel ms, Ms/s.
#
#   ARGS="--scene cornell --streams 64" ROUNDS=2 \
#   VARIANTS="base: units8:BDPT_UNITS=8 pairoff:BDPT_JIT_FLAGS=-DBDPT_RNG_PAIR=0" bash scripts/ab.sh
#   MODE=bench ARGS="--workload caustic8 --no-cpu-baseline" VARIANTS="auto: fused:X=1" bash scripts/ab.sh
#
# A variant is tag:VAR=v[;VAR2=w...] (";" separates assignments; values may hold "," but no
# spaces).  OUT names the result file (gpurun_out/ab.txt).  Every run has its own time limit and
# the session stops at the first failure (no retries on the GPU box).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/ab.txt}
for r in $(seq 1 "${ROUNDS:-2}"); do
  for v in ${VARIANTS:-base:}; do
    tag=${v%%:*}; envs=${v#*:}
    IFS=';' read -r -a assign <<< "$envs"
    if [ "${MODE:-probe}" = bench ]; then
      env "${assign[@]}" timeout -k 10 ${LIMIT:-300} python bench.py ${ARGS:-} > gpurun_out/ab_run.log 2>&1
      rc=$?
      [ $rc -ne 0 ] && { echo "STOP $tag rc=$rc"; tail -5 gpurun_out/ab_run.log; exit $rc; }
      tail -1 gpurun_out/ab_run.log | python3 -c "
import json, sys
d = json.loads(sys.stdin.read())
print('round $r', '$tag', d['config']['pass_streams'], d['ms_per_step'], (d['roofline'] or {}).get('avg_launch_ms'), d['value'])" | tee -a "$OUT"
    else
      env "${assign[@]}" timeout -k 10 ${LIMIT:-150} python scripts/probe_step.py ${ARGS:-} --tag "$tag" > gpurun_out/ab_run.log 2>&1
      rc=$?
      [ $rc -ne 0 ] && { echo "STOP $tag rc=$rc"; tail -5 gpurun_out/ab_run.log; exit $rc; }
      grep '^{' gpurun_out/ab_run.log | tail -1 | python3 -c "
import json, sys
d = json.loads(sys.stdin.read())
print('round $r', d['tag'], d['streams'], d['ms_per_step'], d['kernel_ms'], d['Msamples_s'])" | tee -a "$OUT"
    fi
  done
done
