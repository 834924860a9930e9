set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for v in base default; do
  if [ $v = default ]; then lib=""; else lib=variants/$v/libbdpt.so; fi
  i=0
  for set in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT"; do
    i=$((i+1))
    BDPT_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace -d gpurun_out/pmc_$v/p$i -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/pmc_$v/p$i.log 2>&1 || { echo "fail $v $i"; exit 1; }
  done
  python scripts/pmc_summary.py gpurun_out/pmc_$v path_kernel "p*" > gpurun_out/pmc_$v.txt
done
echo ok
