#!/bin/bash
# round 4 s22: PMC of the pooled path kernel at the caustic N = 1 frame and the N = 8 share
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
SETS=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM GRBM_GUI_ACTIVE"
  "SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT"
  "FETCH_SIZE"
)
for N in 1 8; do
  for i in 0 1 2; do
    rm -rf gpurun_out/s22_n${N}_$i
    BDPT_POOL=${POOLR:-8} BDPT_POOL_GRID=32 timeout -s KILL 120 rocprofv3 --pmc ${SETS[$i]} --kernel-trace -d gpurun_out/s22_n${N}_$i -o run --output-format csv -- \
      python3 scripts/shard_probe.py --scene caustic --passes 128 --strong --ns $N --reps 3 --streams 128 > gpurun_out/s22_n${N}_$i.log 2>&1 || { echo "STOP $N $i"; exit 4; }
    echo "pmc N=$N set $i ok"
  done
done
