#!/bin/bash
# round 5 session 3: streaming (nontemporal) radiance stores and fold loads, fold loads in flight
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "STOP $1 rc=$2"; exit $2; }
P=scripts/probe_step.py
O=gpurun_out/s3_fold_nt.txt
run() { tag=$1; shift; env "$@" timeout -k 10 120 python $P $ARGS --tag $tag >> $O 2>&1 || stop $tag $?; }
for r in 1 2; do
  ARGS="--scene caustic --streams 128"
  run c_base BDPT_POOL=16
  run c_rbufnt BDPT_POOL=16 BDPT_JIT_FLAGS=-DBDPT_RBUF_NT=1
  run c_foldnt BDPT_POOL=16 BDPT_FOLD_KIND=nt
  run c_foldnt8 BDPT_POOL=16 BDPT_FOLD_KIND=nt8
  run c_foldu8 BDPT_POOL=16 BDPT_FOLD_KIND=u8
  run c_both_nt BDPT_POOL=16 BDPT_JIT_FLAGS=-DBDPT_RBUF_NT=1 BDPT_FOLD_KIND=nt
  run c_both_nt8 BDPT_POOL=16 BDPT_JIT_FLAGS=-DBDPT_RBUF_NT=1 BDPT_FOLD_KIND=nt8
  run c_lowprio BDPT_POOL=16 BDPT_FOLD_PRIORITY=low
  ARGS="--scene cornell --streams 64"
  run k_base BDPT_X=0
  run k_both_nt BDPT_JIT_FLAGS=-DBDPT_RBUF_NT=1 BDPT_FOLD_KIND=nt
  run k_both_nt8 BDPT_JIT_FLAGS=-DBDPT_RBUF_NT=1 BDPT_FOLD_KIND=nt8
  run k_foldnt8 BDPT_FOLD_KIND=nt8
done
grep -v amdgpu.ids $O | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['tag'], d['ms_per_step'], d['kernel_ms'], d['Msamples_s'])"
