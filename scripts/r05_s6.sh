#!/bin/bash
# round 5 session 6: where the unit fold loses (timing-only variants without the handover wait /
# without the end-of-unit store wait; unsafe in general, timing only)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "STOP $1 rc=$2"; exit $2; }
P=scripts/probe_step.py
O=gpurun_out/s6_units.txt
run() { tag=$1; shift; env "$@" timeout -k 10 150 python $P $ARGS --tag $tag >> $O 2>&1 || stop $tag $?; }
for r in 1 2; do
  ARGS="--scene cornell --streams 64"
  run k_s64 X=0
  run k_nofold BDPT_ABL_NOFOLD=1 BDPT_JIT_FLAGS=-DBDPT_ABL_NOFOLD=1
  run k_u8 BDPT_UNITS=8
  run k_u8_nowait BDPT_UNITS=8 BDPT_JIT_FLAGS=-DBDPT_UNITS_NOWAIT=1
  run k_u8_noend BDPT_UNITS=8 BDPT_JIT_FLAGS=-DBDPT_UNITS_NOEND=1
  run k_u8_neither BDPT_UNITS=8 BDPT_JIT_FLAGS=-DBDPT_UNITS_NOWAIT=1,-DBDPT_UNITS_NOEND=1
  run k_u2_neither BDPT_UNITS=2 BDPT_JIT_FLAGS=-DBDPT_UNITS_NOWAIT=1,-DBDPT_UNITS_NOEND=1
  run k_u12 BDPT_UNITS=12
done
grep -v amdgpu.ids $O | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['tag'], d['streams'], d['ms_per_step'], d['kernel_ms'], d['Msamples_s'])"
