#!/bin/bash
# Kernel analysis session: shadow-round statistics (instrumented build, precompiled kernels) and
# the VALU instruction mix / stall PMC sets of the default build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
BDPT_LIB=variants/stats/libbdpt.so BDPT_SPECIALIZE=0 timeout -k 10 300 python scripts/shadow_stats.py ${STATS_SCENES:-cornell cornell_glass caustic synthetic64} > gpurun_out/shadow_stats.log 2>&1 || { tail gpurun_out/shadow_stats.log; exit 1; }
cat gpurun_out/shadow_stats.log | grep -v amdgpu.ids
PMC_MIX=1 STEPS=pmc PMC_OUT=mix/p bash scripts/gpu_round.sh
