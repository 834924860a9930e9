#!/bin/bash
# round 5 session 1: smoke, baseline bench lines, weak64 per-band rehearsal, no-fold ablation
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "STOP $1 rc=$2"; exit $2; }
timeout -k 10 200 python -c "import __graft_entry__ as e; e.smoke()" > gpurun_out/s1_smoke.log 2>&1 || stop smoke $?
tail -1 gpurun_out/s1_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/s1_bench_cornell.log 2>&1 || stop bench $?
tail -1 gpurun_out/s1_bench_cornell.log | cut -c1-300
timeout -k 10 300 python bench.py --workload caustic8 --no-cpu-baseline > gpurun_out/s1_bench_caustic8.log 2>&1 || stop caustic8 $?
tail -1 gpurun_out/s1_bench_caustic8.log | cut -c1-300
timeout -k 10 300 python scripts/shard_probe.py --workload weak64 > gpurun_out/s1_weak64_bands.txt 2>&1 || stop weak64 $?
tail -2 gpurun_out/s1_weak64_bands.txt
P=scripts/probe_step.py
for r in 1 2; do
  timeout -k 10 120 python $P --scene cornell --streams 64 --tag base >> gpurun_out/s1_nofold.txt 2>&1 || stop p1 $?
  BDPT_ABL_NOFOLD=1 BDPT_JIT_FLAGS=-DBDPT_ABL_NOFOLD=1 timeout -k 10 120 python $P --scene cornell --streams 64 --tag nofold >> gpurun_out/s1_nofold.txt 2>&1 || stop p2 $?
  timeout -k 10 120 python $P --scene cornell --streams 1 --tag fused >> gpurun_out/s1_nofold.txt 2>&1 || stop p3 $?
  BDPT_JIT_FLAGS=-DBDPT_REGEN_K=64 timeout -k 10 120 python $P --scene cornell --streams 1 --tag fused_lockstep >> gpurun_out/s1_nofold.txt 2>&1 || stop p4 $?
  BDPT_POOL=16 timeout -k 10 120 python $P --scene caustic --streams 128 --tag pools >> gpurun_out/s1_nofold.txt 2>&1 || stop p5 $?
  BDPT_POOL=16 BDPT_ABL_NOFOLD=1 BDPT_JIT_FLAGS=-DBDPT_ABL_NOFOLD=1 timeout -k 10 120 python $P --scene caustic --streams 128 --tag pools_nofold >> gpurun_out/s1_nofold.txt 2>&1 || stop p6 $?
  timeout -k 10 120 python $P --scene caustic --streams 1 --tag fused >> gpurun_out/s1_nofold.txt 2>&1 || stop p7 $?
done
cut -c1-200 gpurun_out/s1_nofold.txt
