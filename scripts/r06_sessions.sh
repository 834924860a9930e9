#!/bin/bash
# The round-6 GPU sessions whose results are under profiles/r06_s<N>_* (one function per
# session; each ran as `gpurun -- bash scripts/r06_sessions.sh s<N>`).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp

pytest_gpu() {   # $1 = log name, rest = pytest selection
  local log=gpurun_out/$1; shift
  timeout -k 10 900 python -u -m pytest "$@" -m gpu -x -q --timeout 300 --timeout-method thread > "$log" 2>&1 \
    || { tail -30 "$log"; return 1; }
  tail -2 "$log"
}

s1() {
  # sin/cos planes (BDPT_SCP): the GPU suite, then bench A/B against the per-vertex fp64 sincos
  pytest_gpu s1_pytest_gpu.log tests || exit 1
  for w in cornell1080 caustic8 weak64; do
    MODE=bench ARGS="--workload $w --no-cpu-baseline" ROUNDS=2 \
      VARIANTS="scp: noscp:BDPT_JIT_FLAGS=-DBDPT_SCP=0" OUT=gpurun_out/s1_ab_scp.txt bash scripts/ab.sh || exit 1
  done
}

s2() {
  # the multi-device tests alone first (s1 aborted in bdpt_create_multi), then the rest as s1
  timeout -k 10 300 python -u -m pytest tests/test_gpu_multi.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/s2_multi.log 2>&1 || { grep -v "^  File" gpurun_out/s2_multi.log | tail -30; exit 1; }
  tail -2 gpurun_out/s2_multi.log
  pytest_gpu s2_pytest_gpu.log tests || exit 1
  for w in cornell1080 caustic8 weak64; do
    MODE=bench ARGS="--workload $w --no-cpu-baseline" ROUNDS=2 \
      VARIANTS="scp: noscp:BDPT_JIT_FLAGS=-DBDPT_SCP=0" OUT=gpurun_out/s2_ab_scp.txt bash scripts/ab.sh || exit 1
  done
}

s3() {
  # sample lists for pooled radiance + sin/cos planes: the GPU suite, then bench A/Bs (prev = the
  # library of commit 2c3421c: sin/cos planes, the [pass][pixel] radiance with a pass bit mask)
  pytest_gpu s3_pytest_gpu.log tests || exit 1
  MODE=bench ARGS="--workload caustic8 --no-cpu-baseline" ROUNDS=2 \
    VARIANTS="lists: prev:BDPT_LIB=gpu_bidirectional_raytracer_amd/libbdpt_prev.so lists_noscp:BDPT_JIT_FLAGS=-DBDPT_SCP=0" \
    OUT=gpurun_out/s3_ab.txt bash scripts/ab.sh || exit 1
  for w in cornell1080 weak64; do
    MODE=bench ARGS="--workload $w --no-cpu-baseline" ROUNDS=2 \
      VARIANTS="scp: noscp:BDPT_JIT_FLAGS=-DBDPT_SCP=0" OUT=gpurun_out/s3_ab.txt bash scripts/ab.sh || exit 1
  done
}

s4() {
  # pools forced (BDPT_POOL=64, whole frame): lists vs prev, wall per step + kernel stats
  ARGS="--scene caustic --streams 128" ROUNDS=2 VARIANTS="lists:BDPT_POOL=64 prev:BDPT_POOL=64;BDPT_LIB=gpu_bidirectional_raytracer_amd/libbdpt_prev.so" \
    OUT=gpurun_out/s4_ab.txt bash scripts/ab.sh || exit 1
  for v in lists prev; do
    lib=""; [ $v = prev ] && lib="BDPT_LIB=gpu_bidirectional_raytracer_amd/libbdpt_prev.so"
    rm -rf gpurun_out/s4_prof_$v
    env BDPT_POOL=64 $lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/s4_prof_$v -o run --output-format csv -- \
      python3 scripts/probe_step.py --scene caustic --streams 128 --reps 5 --tag $v > gpurun_out/s4_prof_$v.log 2>&1 || exit 1
    echo "== $v"; cut -d, -f1-8 gpurun_out/s4_prof_$v/run_kernel_stats.csv | head -6
  done
}

s5() {
  # chunk logs for pooled radiance: pool / config tests first, then the full suite, then A/Bs
  pytest_gpu s5_pytest_pool.log tests/test_gpu_pool.py tests/test_gpu_configs.py -k "pool or every_kernel_mode or config3" || exit 1
  ARGS="--scene caustic --streams 128" ROUNDS=2 VARIANTS="logs:BDPT_POOL=64 prev:BDPT_POOL=64;BDPT_LIB=gpu_bidirectional_raytracer_amd/libbdpt_prev.so" \
    OUT=gpurun_out/s5_ab.txt bash scripts/ab.sh || exit 1
  for v in logs prev; do
    lib=""; [ $v = prev ] && lib="BDPT_LIB=gpu_bidirectional_raytracer_amd/libbdpt_prev.so"
    rm -rf gpurun_out/s5_prof_$v
    env BDPT_POOL=64 BDPT_POOL_OVERLAP=0 $lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/s5_prof_$v -o run --output-format csv -- \
      python3 scripts/probe_step.py --scene caustic --streams 128 --reps 5 --tag $v > gpurun_out/s5_prof_$v.log 2>&1 || exit 1
    echo "== $v (serial launches)"; cut -d, -f1-7 gpurun_out/s5_prof_$v/run_kernel_stats.csv | head -4
  done
  pytest_gpu s5_pytest_gpu.log tests || exit 1
  MODE=bench ARGS="--workload caustic8 --no-cpu-baseline" ROUNDS=2 \
    VARIANTS="logs: prev:BDPT_LIB=gpu_bidirectional_raytracer_amd/libbdpt_prev.so prev_noscp:BDPT_LIB=gpu_bidirectional_raytracer_amd/libbdpt_prev.so;BDPT_JIT_FLAGS=-DBDPT_SCP=0" \
    OUT=gpurun_out/s5_ab.txt bash scripts/ab.sh || exit 1
}

s6() {
  # the multi-device abort (s1, s5: in bdpt_create_multi, intermittent): the test alone, verbose,
  # RCCL warnings on; then the chunk logs (lengths at slot reuse, one-barrier fold) vs prev
  NCCL_DEBUG=WARN timeout -k 10 300 python -u -m pytest tests/test_gpu_multi.py -m gpu -x -v -s --timeout 120 --timeout-method thread > gpurun_out/s6_multi.log 2>&1 || { grep -v "^  File" gpurun_out/s6_multi.log | tail -40; exit 1; }
  tail -2 gpurun_out/s6_multi.log
  pytest_gpu s6_pytest_pool.log tests/test_gpu_pool.py tests/test_gpu_configs.py -k "pool or every_kernel_mode or config3" || exit 1
  ARGS="--scene caustic --streams 128" ROUNDS=2 VARIANTS="logs64:BDPT_POOL=64 logs32:BDPT_POOL=32 prev:BDPT_POOL=64;BDPT_LIB=gpu_bidirectional_raytracer_amd/libbdpt_prev.so" \
    OUT=gpurun_out/s6_ab.txt bash scripts/ab.sh || exit 1
  for v in logs prev; do
    lib=""; [ $v = prev ] && lib="BDPT_LIB=gpu_bidirectional_raytracer_amd/libbdpt_prev.so"
    rm -rf gpurun_out/s6_prof_$v
    env BDPT_POOL=64 BDPT_POOL_OVERLAP=0 $lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/s6_prof_$v -o run --output-format csv -- \
      python3 scripts/probe_step.py --scene caustic --streams 128 --reps 5 --tag $v > gpurun_out/s6_prof_$v.log 2>&1 || exit 1
    echo "== $v (serial launches)"; cut -d, -f1-7 gpurun_out/s6_prof_$v/run_kernel_stats.csv | head -4
  done
}

s7() {
  # the multi-device abort: a stress loop of bdpt_create_multi([0]) with RCCL warnings on, then the
  # full suite with output uncaptured (-s) so an abort's stderr is kept; then the reverted pools
  NCCL_DEBUG=WARN timeout -k 10 240 python -u scripts/multi_stress.py --n 60 > gpurun_out/s7_stress.log 2>&1 || { tail -30 gpurun_out/s7_stress.log; exit 1; }
  tail -2 gpurun_out/s7_stress.log
  NCCL_DEBUG=WARN timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/s7_pytest_gpu.log 2>&1 || { grep -v "^  File" gpurun_out/s7_pytest_gpu.log | tail -60; exit 1; }
  grep -c PASSED gpurun_out/s7_pytest_gpu.log; tail -1 gpurun_out/s7_pytest_gpu.log
}

s8() {
  # final build: the multi tests (RCCL group case in a child), A/Bs (sin/cos planes on caustic8,
  # the release/acquire handover variant of units), caustic8 strong-scaling shares, final benches
  pytest_gpu s8_pytest_multi.log tests/test_gpu_multi.py || exit 1
  MODE=bench ARGS="--workload caustic8 --no-cpu-baseline" ROUNDS=2 \
    VARIANTS="scp: noscp:BDPT_JIT_FLAGS=-DBDPT_SCP=0" OUT=gpurun_out/s8_ab_scp_caustic8.txt bash scripts/ab.sh || exit 1
  ARGS="--scene cornell --streams 64" ROUNDS=2 \
    VARIANTS="units:BDPT_UNITS=8 units_fence:BDPT_UNITS=8;BDPT_JIT_FLAGS=-DBDPT_UNITS_FENCE=1" OUT=gpurun_out/s8_ab_fence.txt bash scripts/ab.sh || exit 1
  timeout -k 10 500 python scripts/shard_probe.py --scene caustic --passes 128 --strong --reps 20 > gpurun_out/s8_caustic_strong.txt 2>&1 || { tail -20 gpurun_out/s8_caustic_strong.txt; exit 1; }
  tail -8 gpurun_out/s8_caustic_strong.txt
  for w in cornell1080 caustic8 weak64; do
    timeout -k 10 400 python bench.py --workload $w > gpurun_out/s8_bench_$w.log 2>&1 || { tail -20 gpurun_out/s8_bench_$w.log; exit 1; }
    grep '^{' gpurun_out/s8_bench_$w.log | tail -1 > gpurun_out/s8_bench_$w.json
    python3 -c "import json; d=json.load(open('gpurun_out/s8_bench_$w.json')); print('$w', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('traffic_over_model'), d.get('speedup_vs_cpu_node_estimate'))"
  done
}

s9() {
  # the final build (sin/cos planes off in the pool build): GPU suite, caustic8 bench, then
  # per-workload rocprof stats + PMC records
  pytest_gpu s9_pytest_gpu.log tests || exit 1
  timeout -k 10 400 python bench.py --workload caustic8 > gpurun_out/s9_bench_caustic8.log 2>&1 || { tail -20 gpurun_out/s9_bench_caustic8.log; exit 1; }
  grep '^{' gpurun_out/s9_bench_caustic8.log | tail -1 > gpurun_out/s9_bench_caustic8.json
  python3 -c "import json; d=json.load(open('gpurun_out/s9_bench_caustic8.json')); print('caustic8', d['value'], d['ms_per_step'], d['roofline']['frac'])"
  WORKLOADS="cornell1080:64:cornell1080:BDPT_UNITS=8 cornell1080:64:cornell1080s64:BDPT_UNITS=0 caustic8:128:caustic8:BDPT_POOL=16 weak64:32" \
    bash scripts/profile_workloads.sh
}

s10() {
  # the driver's other entry points on the final build: smoke(), multi-rank rehearsals (gloo,
  # ranks sharing the GPU), an in-process two-device group on one GPU (peer copies)
  timeout -k 10 300 python -c "import __graft_entry__ as e; e.smoke()" > gpurun_out/s10_smoke.log 2>&1 || { tail -20 gpurun_out/s10_smoke.log; exit 1; }
  tail -1 gpurun_out/s10_smoke.log
  NS="2 4" WORKLOADS="cornell1080 caustic8" STEPS_N=4 bash scripts/rehearse.sh || exit 1
  for w in cornell1080 caustic8; do for n in 2 4; do grep '^{' gpurun_out/rehearse_${w}_$n.log | tail -1 > gpurun_out/s10_rehearse_${w}_$n.json; done; done
  timeout -k 10 300 python bench.py --gpus 2 --devices 0,0 --steps 5 --no-cpu-baseline > gpurun_out/s10_inproc.log 2>&1 || { tail -20 gpurun_out/s10_inproc.log; exit 1; }
  grep '^{' gpurun_out/s10_inproc.log | tail -1 > gpurun_out/s10_inproc.json
  for f in gpurun_out/s10_rehearse_*.json gpurun_out/s10_inproc.json; do
    python3 -c "
import json; d=json.load(open('$f'))
print('$f', d['n_gpus'], d['value'], d['reduce_backend'], 'modes_agree', d.get('modes_agree'), d.get('rccl_version'))"
  done
}

s11() {
  # pool kernel occupancy: 7 waves/SIMD (6 VGPRs spilled) against the default 6, caustic8 bench
  MODE=bench ARGS="--workload caustic8 --no-cpu-baseline" ROUNDS=2 \
    VARIANTS="w6: w7:BDPT_JIT_WAVES=7;BDPT_JIT_SCRATCH_OK=1" OUT=gpurun_out/s11_ab_waves.txt bash scripts/ab.sh || exit 1
}

s12() {
  # other scenes on the final build (BVH scenes take the precompiled kernels with the sin/cos
  # planes), and the default bench line with the round-6 PMC records
  for sc in complex mod_cornell cornell_glass; do
    timeout -k 10 400 python bench.py --scene $sc --no-cpu-baseline --steps 5 > gpurun_out/s12_bench_$sc.log 2>&1 || { tail -20 gpurun_out/s12_bench_$sc.log; exit 1; }
    grep '^{' gpurun_out/s12_bench_$sc.log | tail -1 > gpurun_out/s12_bench_$sc.json
    python3 -c "import json; d=json.load(open('gpurun_out/s12_bench_$sc.json')); print('$sc', d['value'], d['ms_per_step'], d['config']['traversal'], d['roofline'] and d['roofline']['kernel_features'])"
  done
  timeout -k 10 400 python bench.py > gpurun_out/s12_bench_default.log 2>&1 || { tail -20 gpurun_out/s12_bench_default.log; exit 1; }
  grep '^{' gpurun_out/s12_bench_default.log | tail -1 > gpurun_out/s12_bench_default.json
  python3 -c "import json; d=json.load(open('gpurun_out/s12_bench_default.json')); r=d['roofline']; print('default', d['value'], r['frac'], r['traffic'], r['traffic_over_model'], r.get('valu_busy_pmc'), d.get('speedup_vs_cpu_node_estimate'))"
}

s13() {
  # the sin/cos planes in the precompiled BVH kernels: this build against one with BDPT_SCP=0
  # (make variant NAME=noscp EXTRA_HIPFLAGS=-DBDPT_SCP=0)
  for sc in complex mod_cornell; do
    MODE=bench ARGS="--scene $sc --no-cpu-baseline --steps 5" ROUNDS=2 \
      VARIANTS="scp: noscp:BDPT_LIB=variants/noscp/libbdpt.so" OUT=gpurun_out/s13_ab_scp_bvh.txt bash scripts/ab.sh || exit 1
  done
}

s14() {
  # the final tree: the GPU suite once more (the driver's round-end command) and smoke()
  pytest_gpu s14_pytest_gpu.log tests || exit 1
  timeout -k 10 300 python -c "import __graft_entry__ as e; e.smoke()" > gpurun_out/s14_smoke.log 2>&1 || { tail -20 gpurun_out/s14_smoke.log; exit 1; }
  tail -1 gpurun_out/s14_smoke.log
}

s15() {
  # do transcendental / fp64 instructions take fp32 VALU issue cycles? (scripts/valu_overlap.hip)
  timeout -k 10 120 ./scripts/valu_overlap > gpurun_out/s15_valu_overlap.txt 2>&1 || { tail -5 gpurun_out/s15_valu_overlap.txt; exit 1; }
  cat gpurun_out/s15_valu_overlap.txt
}

s16() {
  # the sin/cos pairs loaded at the top of their own segment (BDPT_SCP_LATE) against one segment
  # ahead (default) and no planes
  for w in cornell1080 weak64; do
    MODE=bench ARGS="--workload $w --no-cpu-baseline" ROUNDS=2 \
      VARIANTS="early: late:BDPT_JIT_FLAGS=-DBDPT_SCP_LATE=1 noscp:BDPT_JIT_FLAGS=-DBDPT_SCP=0" \
      OUT=gpurun_out/s16_ab_scp_late.txt bash scripts/ab.sh || exit 1
  done
}

s17() {
  # the 1080p whole-frame mode test, now against the oracle over every pixel
  pytest_gpu s17_pytest_wholeframe.log tests/test_gpu_configs.py -k whole_frame --durations=5 || exit 1
  grep -A8 "slowest" gpurun_out/s17_pytest_wholeframe.log
}

s18() {
  # the display entry points on the GPU (no GL context on the node: refusal + bit-exact render after)
  pytest_gpu s18_pytest_display.log tests/test_display.py tests/test_gpu_parity.py || exit 1
}

s19() {
  # configs[3] against the oracle over the whole frame at 4096 spp; the whole-frame mode test with
  # cornell_glass added
  pytest_gpu s19_pytest_configs.log tests/test_gpu_configs.py --durations=10 || exit 1
  grep -A12 "slowest" gpurun_out/s19_pytest_configs.log
}

s20() {
  # the final tree (display entry points, whole-frame config tests): GPU suite, smoke, default bench
  pytest_gpu s20_pytest_gpu.log tests || exit 1
  timeout -k 10 300 python -c "import __graft_entry__ as e; e.smoke()" > gpurun_out/s20_smoke.log 2>&1 || { tail -20 gpurun_out/s20_smoke.log; exit 1; }
  tail -1 gpurun_out/s20_smoke.log
  timeout -k 10 400 python bench.py > gpurun_out/s20_bench_default.log 2>&1 || { tail -20 gpurun_out/s20_bench_default.log; exit 1; }
  grep '^{' gpurun_out/s20_bench_default.log | tail -1 > gpurun_out/s20_bench_default.json
  python3 -c "import json; d=json.load(open('gpurun_out/s20_bench_default.json')); r=d['roofline']; print('default', d['value'], d['ms_per_step'], r['frac'], r['avg_launch_ms'], d.get('speedup_vs_cpu_node_estimate'))"
}

s21() {
  # every reference scene on the final build (bench.py, 1921x1081, 32 passes per step)
  timeout -k 10 1000 bash scripts/scenes_sweep.sh || exit 1
}

s22() {
  # emitter tests skipped in VLP-only shadow rounds (BDPT_VAC_SKIP): parity first, then A/B
  pytest_gpu s22_pytest_parity.log tests/test_gpu_parity.py tests/test_gpu_fuzz.py || exit 1
  for w in cornell1080 weak64 caustic8; do
    MODE=bench ARGS="--workload $w --no-cpu-baseline" ROUNDS=2 \
      VARIANTS="skip: noskip:BDPT_JIT_FLAGS=-DBDPT_VAC_SKIP=0" \
      OUT=gpurun_out/s22_ab_vac_skip.txt bash scripts/ab.sh || exit 1
  done
}

s23() {
  # VLP-only part-full shadow rounds over the non-emitters' list (BDPT_VAC_LIST) on top of the
  # emitter skip in full rounds (BDPT_VAC_SKIP): parity first, then A/B
  pytest_gpu s23_pytest_parity.log tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_configs.py -k "not config4" || exit 1
  for w in cornell1080 weak64 caustic8; do
    MODE=bench ARGS="--workload $w --no-cpu-baseline" ROUNDS=2 \
      VARIANTS="list: skiponly:BDPT_JIT_FLAGS=-DBDPT_VAC_LIST=0 none:BDPT_JIT_FLAGS=-DBDPT_VAC_LIST=0,-DBDPT_VAC_SKIP=0" \
      OUT=gpurun_out/s23_ab_vac_list.txt bash scripts/ab.sh || exit 1
  done
}

s24() {
  # the list kept out of the pool build and the precompiled instances: full GPU suite, then A/B
  pytest_gpu s24_pytest_gpu.log tests || exit 1
  for w in cornell1080 caustic8 weak64; do
    MODE=bench ARGS="--workload $w --no-cpu-baseline" ROUNDS=2 \
      VARIANTS="list: skiponly:BDPT_JIT_FLAGS=-DBDPT_VAC_LIST=0" \
      OUT=gpurun_out/s24_ab_vac_list.txt bash scripts/ab.sh || exit 1
  done
}

s25() {
  # per-section shares of the cornell1080 kernel after the VLP-round changes
  RUNS="cornell1080:64" bash scripts/section_profile.sh || exit 1
}

s26() {
  # final-build rocprof stats + PMC records, cornell1080 in each mode the auto choice can take
  WORKLOADS="cornell1080:64:cornell1080:BDPT_UNITS=8 cornell1080:64:cornell1080s64:BDPT_UNITS=0 cornell1080:32:cornell1080s32:BDPT_UNITS=0" \
    bash scripts/profile_workloads.sh
}

s27() {
  # final-build rocprof stats + PMC records: caustic8 (pools), weak64 at both stream counts
  WORKLOADS="caustic8:128:caustic8:BDPT_POOL=16 weak64:32 weak64:16:weak64s16:BDPT_UNITS=0" \
    bash scripts/profile_workloads.sh
}

s28() {
  # the final tree as the driver runs it: GPU suite, smoke, default bench; then the other
  # workloads' bench lines with the CPU leg
  pytest_gpu s28_pytest_gpu.log tests || exit 1
  timeout -k 10 300 python -c "import __graft_entry__ as e; e.smoke()" > gpurun_out/s28_smoke.log 2>&1 || { tail -20 gpurun_out/s28_smoke.log; exit 1; }
  tail -1 gpurun_out/s28_smoke.log
  for w in default caustic8 weak64; do
    a=""; [ $w != default ] && a="--workload $w"
    timeout -k 10 400 python bench.py $a > gpurun_out/s28_bench_$w.log 2>&1 || { tail -20 gpurun_out/s28_bench_$w.log; exit 1; }
    grep '^{' gpurun_out/s28_bench_$w.log | tail -1 > gpurun_out/s28_bench_$w.json
    python3 -c "import json; d=json.load(open('gpurun_out/s28_bench_$w.json')); r=d['roofline']; print('$w', d['value'], d['ms_per_step'], r['frac'], r['avg_launch_ms'], r.get('traffic_over_model'), r.get('valu_busy_pmc'), d.get('speedup_vs_cpu_node_estimate'))"
  done
}

s29() {
  # the lane-group rule of part-full shadow rounds (BDPT_LG_RULE): parity first, then A/B
  pytest_gpu s29_pytest_parity.log tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_pool.py || exit 1
  for w in cornell1080 caustic8 weak64; do
    MODE=bench ARGS="--workload $w --no-cpu-baseline" ROUNDS=2 \
      VARIANTS="rule: old:BDPT_JIT_FLAGS=-DBDPT_LG_RULE=0" \
      OUT=gpurun_out/s29_ab_lg_rule.txt bash scripts/ab.sh || exit 1
  done
}

s31() {
  # the VLP-round changes on the two-light and mirror scenes (sweep spread check), one session
  for sc in cornell_2luci synthetic64 hall_of_mirrors; do
    MODE=bench ARGS="--scene $sc --no-cpu-baseline --passes 32 --steps 10" ROUNDS=2 \
      VARIANTS="final: off:BDPT_JIT_FLAGS=-DBDPT_VAC_LIST=0,-DBDPT_VAC_SKIP=0,-DBDPT_LG_RULE=0" \
      OUT=gpurun_out/s31_ab_scenes.txt bash scripts/ab.sh || exit 1
  done
}

s32() {
  # cornell_2luci (two emitters): which of the three shadow-round changes costs, fixed 16 streams
  for sc in cornell_2luci hall_of_mirrors; do
    MODE=bench ARGS="--scene $sc --no-cpu-baseline --passes 32 --steps 10 --streams 16" ROUNDS=2 \
      VARIANTS="final: noskip:BDPT_JIT_FLAGS=-DBDPT_VAC_SKIP=0 nolist:BDPT_JIT_FLAGS=-DBDPT_VAC_LIST=0 oldlg:BDPT_JIT_FLAGS=-DBDPT_LG_RULE=0 off:BDPT_JIT_FLAGS=-DBDPT_VAC_LIST=0,-DBDPT_VAC_SKIP=0,-DBDPT_LG_RULE=0" \
      OUT=gpurun_out/s32_ab_flags.txt bash scripts/ab.sh || exit 1
  done
}

s33() {
  # the non-emitters' list made opt-in (BDPT_VAC_LIST=1): parity, cornell1080 / cornell_2luci A/B,
  # then cornell1080's profiles on the default build
  pytest_gpu s33_pytest_parity.log tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_configs.py -k "not config4" || exit 1
  MODE=bench ARGS="--workload cornell1080 --no-cpu-baseline" ROUNDS=2 \
    VARIANTS="default: list:BDPT_VAC_LIST=1" OUT=gpurun_out/s33_ab_list_optin.txt bash scripts/ab.sh || exit 1
  MODE=bench ARGS="--scene cornell_2luci --no-cpu-baseline --passes 32 --steps 10 --streams 16" ROUNDS=2 \
    VARIANTS="default: list:BDPT_VAC_LIST=1" OUT=gpurun_out/s33_ab_list_optin.txt bash scripts/ab.sh || exit 1
  WORKLOADS="cornell1080:64:cornell1080:BDPT_UNITS=8 cornell1080:64:cornell1080s64:BDPT_UNITS=0 cornell1080:32:cornell1080s32:BDPT_UNITS=0" \
    bash scripts/profile_workloads.sh
}

s34() {
  # the tree rebuilt in a fresh container (same sources as s28): GPU suite, smoke, default bench
  pytest_gpu s34_pytest_gpu.log tests || exit 1
  timeout -k 10 300 python -c "import __graft_entry__ as e; e.smoke()" > gpurun_out/s34_smoke.log 2>&1 || { tail -20 gpurun_out/s34_smoke.log; exit 1; }
  tail -1 gpurun_out/s34_smoke.log
  timeout -k 10 400 python bench.py > gpurun_out/s34_bench_default.log 2>&1 || { tail -20 gpurun_out/s34_bench_default.log; exit 1; }
  grep '^{' gpurun_out/s34_bench_default.log | tail -1
}

"$@"
