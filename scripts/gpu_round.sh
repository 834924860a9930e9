#!/bin/bash
# One GPU-box session: parity tests, bench, rocprofv3 kernel trace.  Each GPU step has its own
# time limit; a crash/abort/timeout (exit >= 124 or signal) stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ok_or_stop() {  # $1 = exit code, $2 = step name; test failures (1) continue, faults stop
  if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "STOP after $2 (exit $1)"; exit "$1"; fi
}
STEPS="${STEPS:-tests bench prof}"
if [ -n "${PMC_MIX:-}" ]; then PMC_SETS=(
  "SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64"
  "SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FLOPS_FP32_TRANS SQ_INSTS_VALU_IOPS SQ_INSTS_VALU"
  "SQ_INSTS_LDS_LOAD SQ_INSTS_LDS_STORE SQ_INSTS_BRANCH SQ_INST_CYCLES_SALU SQ_INST_CYCLES_SMEM SQ_INSTS_VSKIPPED SQ_INSTS_SMEM SQ_INSTS_SALU"
  "SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
); else PMC_SETS=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM GRBM_GUI_ACTIVE"
  "SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT"
  "FETCH_SIZE"
  "WRITE_SIZE"
  "TCC_HIT_sum TCC_MISS_sum"
); fi
for s in $STEPS; do
  case "$s" in
  tests)
    timeout -k 10 900 python -u -m pytest tests -m gpu -v -rA --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
    rc=$?; tail -30 gpurun_out/pytest_gpu.log; ok_or_stop $rc tests ;;
  smoke)
    timeout -k 10 300 python -c "import __graft_entry__ as e; e.smoke()" > gpurun_out/smoke.log 2>&1
    rc=$?; cat gpurun_out/smoke.log; ok_or_stop $rc smoke ;;
  bench)
    timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
    rc=$?; tail -5 gpurun_out/bench.log; ok_or_stop $rc bench ;;
  prof)
    rm -rf gpurun_out/prof
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
        python3 bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/prof.log 2>&1
    rc=$?; tail -3 gpurun_out/prof.log; find gpurun_out/prof -name "*stats*" | head; ok_or_stop $rc prof ;;
  scenes)
    for sc in ${SCENES_LIST:-cornell cornell_glass caustic simple synthetic64}; do
      timeout -k 10 300 python bench.py --no-cpu-baseline --scene $sc ${BENCH_ARGS:-} > gpurun_out/scene_$sc.log 2>&1
      rc=$?; echo "scene $sc rc=$rc $(tail -1 gpurun_out/scene_$sc.log | cut -c1-90)"
      python -c "import json; d=json.loads(open('gpurun_out/scene_$sc.log').read().strip().splitlines()[-1]); print('   ', d['value'], 'Msamples/s', d['device_ms_per_step'], 'ms/step', 'valu TF', d['roofline']['achieved'] if d['roofline'] else None)" || true
      ok_or_stop $rc scene_$sc
    done ;;
  workloads)
    for w in ${WORKLOADS_LIST:-caustic8 weak64}; do
      timeout -k 10 400 python bench.py --workload $w --cpu-seconds 6 > gpurun_out/wl_$w.log 2>&1
      rc=$?; echo "workload $w rc=$rc"; tail -1 gpurun_out/wl_$w.log | cut -c1-400; ok_or_stop $rc wl_$w
    done ;;
  inproc)
    # bench.py --gpus N without torchrun: one in-process multi-device context (rehearsed on one
    # GPU with --devices 0,0: two shards, peer-copy reduce), then --gpus 2 must refuse on 1 GPU
    timeout -k 10 300 python bench.py --gpus 2 --devices 0,0 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/inproc.log 2>&1
    rc=$?; tail -1 gpurun_out/inproc.log | cut -c1-600; ok_or_stop $rc inproc
    timeout -k 10 120 python bench.py --gpus 2 --steps 2 > gpurun_out/refuse.log 2>&1
    rc=$?; echo "--gpus 2 on this box: exit $rc: $(tail -1 gpurun_out/refuse.log)"
    [ $rc -eq 1 ] || { echo "STOP refuse (expected exit 1)"; exit 3; } ;;
  profile)
    timeout -k 10 1500 bash scripts/profile_workloads.sh > gpurun_out/profile.log 2>&1
    rc=$?; tail -20 gpurun_out/profile.log; ok_or_stop $rc profile ;;
  shard)
    timeout -k 10 400 python scripts/shard_probe.py ${SHARD_ARGS:-} > gpurun_out/shard_probe.log 2>&1
    rc=$?; cat gpurun_out/shard_probe.log | tail -12; ok_or_stop $rc shard ;;
  calib)
    # FETCH_SIZE / WRITE_SIZE calibration on known byte counts (scripts/pmc_calib.hip)
    [ -x scripts/pmc_calib ] || /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -o scripts/pmc_calib scripts/pmc_calib.hip
    for c in FETCH_SIZE WRITE_SIZE; do
      rm -rf gpurun_out/calib_$c
      timeout -k 10 180 rocprofv3 --pmc $c --kernel-trace -d gpurun_out/calib_$c -o run --output-format csv -- \
          ./scripts/pmc_calib > gpurun_out/calib_$c.log 2>&1
      rc=$?; echo "calib $c rc=$rc"; ok_or_stop $rc calib_$c
    done
    cp gpurun_out/calib_FETCH_SIZE.log gpurun_out/calib_bytes.jsonl ;;
  pmc)
    rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
    i=0
    for set in "${PMC_SETS[@]}"; do
      i=$((i+1)); P=gpurun_out/${PMC_OUT:-pmc}; rm -rf $P$i; mkdir -p $(dirname $P)
      timeout -s KILL 240 rocprofv3 --pmc $set --kernel-trace -d $P$i -o run --output-format csv -- \
          python3 bench.py --no-cpu-baseline --steps 4 --warmup 1 ${BENCH_ARGS:-} > $P$i.log 2>&1
      rc=$?; echo "pmc set $i ($set): rc=$rc"; tail -1 $P$i.log; ok_or_stop $rc pmc$i
    done ;;
  esac
done
echo ALL_DONE
