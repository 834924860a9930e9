#!/bin/bash
# Per-workload profiles on the GPU box: for each bench.py workload, one rocprofv3 kernel-trace
# --stats run of the default bench command and the PMC passes (separate runs, MI355X_MICROARCH.md
# "HBM") with the pass-stream mode the default run settles on (S = half the launch's passes: two
# passes per lane; 1: fused);
# the last two passes split the VALU instructions by class (scripts/valu_weighted.py).
#   WORKLOADS="cornell1080:64 caustic8:1 weak64:32" bash scripts/profile_workloads.sh
# An entry w:S:name profiles workload w at S streams under the output name `name` (e.g.
# cornell1080:32:cornell1080s32 next to cornell1080:64, for both outcomes of the auto mode);
# w:S:name:VAR=value sets an environment variable for the PMC passes (caustic8:128:caustic8:
# BDPT_POOL=16 = the pixel pools the auto mode keeps for caustic8).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
export BDPT_JIT_CACHE=$(mktemp -d /tmp/bdpt-jit-prof.XXXXXX)     # one compile per scene, shared
stop() { echo "STOP $1 (exit $2)"; exit "$2"; }
PMC_SETS=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM GRBM_GUI_ACTIVE"
  "SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT"
  "FETCH_SIZE"
  "WRITE_SIZE"
  "TCC_HIT_sum TCC_MISS_sum"
  "SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 GRBM_GUI_ACTIVE"
  "SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE"
)
for ws in ${WORKLOADS:-cornell1080:64 caustic8:128:caustic8:BDPT_POOL=16 weak64:32}; do
  IFS=: read -r w S name penv <<< "$ws"; name=${name:-$w}; penv=${penv:-BDPT_PROFILE_ENV=1}
  steps=${STEPS_STATS:-10}
  [ "$w" = weak64 ] && steps=${STEPS_STATS64:-6}
  rm -rf gpurun_out/prof_$name
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$name -o run --output-format csv -- \
      python3 bench.py --workload $w --no-cpu-baseline --steps $steps --warmup 3 > gpurun_out/prof_$name.log 2>&1 || stop "stats $name" $?
  echo "stats $name: $(grep '^{' gpurun_out/prof_$name.log | tail -1 | cut -c1-200)"
  i=0
  for set in "${PMC_SETS[@]}"; do
    i=$((i+1)); rm -rf gpurun_out/pmc_${name}_$i
    env $penv timeout -s KILL 240 rocprofv3 --pmc $set --kernel-trace -d gpurun_out/pmc_${name}_$i -o run --output-format csv -- \
        python3 bench.py --workload $w --no-cpu-baseline --no-smt-probe --steps 4 --warmup 1 --streams $S > gpurun_out/pmc_${name}_$i.log 2>&1 || stop "pmc $name $i" $?
    echo "pmc $name set $i ok"
  done
done
echo PROFILE_DONE
