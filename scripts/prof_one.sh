#!/bin/bash
# One workload at one stream setting: rocprofv3 kernel-trace --stats plus selected PMC passes
# (separate runs).  NAME=x W=caustic8 S=16 SETS="1 2 3" bash scripts/prof_one.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
export BDPT_JIT_CACHE=$(mktemp -d /tmp/bdpt-jit-prof.XXXXXX)
PMC_SETS=(
  ""
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM GRBM_GUI_ACTIVE"
  "SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT"
  "FETCH_SIZE"
  "WRITE_SIZE"
  "TCC_HIT_sum TCC_MISS_sum"
)
n=${NAME:-$W}
rm -rf gpurun_out/prof_$n
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$n -o run --output-format csv -- \
    python3 bench.py --workload $W --no-cpu-baseline --tail-seconds 0 --steps ${STEPS:-10} --warmup 3 --streams $S ${EXTRA:-} > gpurun_out/prof_$n.log 2>&1 || { echo "STOP stats $?"; exit 3; }
echo "stats $n: $(grep '^{' gpurun_out/prof_$n.log | tail -1 | cut -c1-160)"
for i in ${SETS:-}; do
  rm -rf gpurun_out/pmc_${n}_$i
  timeout -s KILL 240 rocprofv3 --pmc ${PMC_SETS[$i]} --kernel-trace -d gpurun_out/pmc_${n}_$i -o run --output-format csv -- \
      python3 bench.py --workload $W --no-cpu-baseline --tail-seconds 0 --steps 4 --warmup 1 --streams $S ${EXTRA:-} > gpurun_out/pmc_${n}_$i.log 2>&1 || { echo "STOP pmc $i"; exit 4; }
  echo "pmc $n set $i ok"
done
