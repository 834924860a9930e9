#!/bin/bash
# round 5 session 4: is the fused kernel's deficit on cornell its launch tail?  (1080p vs 4K frame)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "STOP $1 rc=$2"; exit $2; }
P=scripts/probe_step.py
O=gpurun_out/s4_tail.txt
run() { tag=$1; shift; env "$@" timeout -k 10 150 python $P $ARGS --tag $tag >> $O 2>&1 || stop $tag $?; }
for r in 1 2; do
  ARGS="--scene cornell --passes 128 --streams 64"; run k1080_s64 X=0
  ARGS="--scene cornell --passes 128 --streams 1"; run k1080_fused X=0
  ARGS="--scene cornell --passes 32 --streams 16 --width 3841 --height 2161"; run k4k_s16 X=0
  ARGS="--scene cornell --passes 32 --streams 1 --width 3841 --height 2161"; run k4k_fused X=0
  ARGS="--scene caustic --passes 128 --streams 1"; run c1080_fused X=0
  ARGS="--scene caustic --passes 32 --streams 1 --width 3841 --height 2161"; run c4k_fused X=0
  ARGS="--scene caustic --passes 32 --streams 32 --width 3841 --height 2161"; run c4k_pools BDPT_POOL=16
done
grep -v amdgpu.ids $O | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['tag'], d['streams'], d['ms_per_step'], d['kernel_ms'], d['Msamples_s'])"
