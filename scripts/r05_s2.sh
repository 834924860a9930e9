#!/bin/bash
# round 5 session 2: split the no-fold ablation into its two halves (stores vs fold kernel)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "STOP $1 rc=$2"; exit $2; }
P=scripts/probe_step.py
O=gpurun_out/s2_split.txt
for r in 1 2; do
  BDPT_POOL=16 timeout -k 10 120 python $P --scene caustic --streams 128 --tag pools >> $O 2>&1 || stop p1 $?
  BDPT_POOL=16 BDPT_JIT_FLAGS=-DBDPT_ABL_NOFOLD=1 timeout -k 10 120 python $P --scene caustic --streams 128 --tag pools_nostore >> $O 2>&1 || stop p2 $?
  BDPT_POOL=16 BDPT_ABL_NOFOLD=1 timeout -k 10 120 python $P --scene caustic --streams 128 --tag pools_nofoldkernel >> $O 2>&1 || stop p3 $?
  timeout -k 10 120 python $P --scene cornell --streams 64 --tag s64 >> $O 2>&1 || stop p4 $?
  BDPT_JIT_FLAGS=-DBDPT_ABL_NOFOLD=1 timeout -k 10 120 python $P --scene cornell --streams 64 --tag s64_nostore >> $O 2>&1 || stop p5 $?
  BDPT_ABL_NOFOLD=1 timeout -k 10 120 python $P --scene cornell --streams 64 --tag s64_nofoldkernel >> $O 2>&1 || stop p6 $?
done
grep -v amdgpu.ids $O | cut -c1-170
