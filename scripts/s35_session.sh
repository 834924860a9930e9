#!/bin/bash
# round 4 s35: section profile of the fused vs pooled kernel on caustic8, and the occupancy PMC
# (set 0 of s22) of the pooled kernel at the N = 1 frame and the N = 8 share with interleaved passes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
BDPT_POOL=16 RUNS="caustic8:1 caustic8:128" timeout -k 10 600 bash scripts/section_profile.sh > gpurun_out/s35_sections.log 2>&1 || exit 3
SET="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM GRBM_GUI_ACTIVE"
for N in 1 8; do
  rm -rf gpurun_out/s35_n$N
  BDPT_POOL=8 BDPT_POOL_GRID=32 timeout -s KILL 120 rocprofv3 --pmc $SET --kernel-trace -d gpurun_out/s35_n$N -o run --output-format csv -- \
    python3 scripts/shard_probe.py --scene caustic --passes 128 --strong --ns $N --reps 3 --streams 128 > gpurun_out/s35_n$N.log 2>&1 || { echo "STOP pmc $N"; exit 4; }
  echo "pmc N=$N ok"
done
