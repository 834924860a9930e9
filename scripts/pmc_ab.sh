#!/bin/bash
# PMC comparison of run-time variants in one GPU session (experiments):
#   VARIANTS="BDPT_JIT_FLAGS=-DBDPT_IKEY=1|" [PMCSET="..."] bash scripts/pmc_ab.sh
# then python scripts/pmc_summary.py gpurun_out path_kernel "pmcab_v1_*"
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out; export TMPDIR=/tmp
export BDPT_JIT_CACHE=$(mktemp -d /tmp/bdpt-jit-ab.XXXXXX)
IFS='|' read -r -a VS <<< "${VARIANTS}"
SET="${PMCSET:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE}"
k=0
for v in "${VS[@]}"; do
  k=$((k+1)); P=gpurun_out/pmcab_v${k}_1; rm -rf $P
  env $v timeout -s KILL 120 rocprofv3 --pmc $SET --kernel-trace -d $P -o run --output-format csv -- \
      python3 bench.py --no-cpu-baseline --steps 4 --warmup 3 --streams -1 ${BENCH_ARGS:-} > $P.log 2>&1
  rc=$?; echo "v$k [$v] rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $P.log; exit $rc; fi
done
echo PMC_DONE
