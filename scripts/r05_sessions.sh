#!/bin/bash
# The round-5 GPU sessions whose results are under profiles/r05_s<N>_* (one function per
# session; each ran as `gpurun -- bash scripts/r05_sessions.sh s<N>`).  Later rounds: use
# scripts/ab.sh for A/Bs and add a session here only when its output is committed.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp

s9() {
  # round 5 session 9: per-workload rocprof stats + PMC records (units for cornell1080), weak64 bench
  cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
  mkdir -p gpurun_out
  export TMPDIR=/tmp
  WORKLOADS="cornell1080:64:cornell1080:BDPT_UNITS=8 caustic8:128:caustic8:BDPT_POOL=16 weak64:32" bash scripts/profile_workloads.sh
}

s10() {
  timeout -k 10 300 python -u -m pytest tests/test_gpu_units.py tests/test_gpu_parity.py -k "units or auto_streams" -x -q --timeout 120 --timeout-method thread > gpurun_out/s10_pytest.log 2>&1 || { tail -20 gpurun_out/s10_pytest.log; exit 1; }
  tail -2 gpurun_out/s10_pytest.log
  NS="2 4" WORKLOADS="cornell1080" STEPS_N=4 bash scripts/rehearse.sh || exit 1
  for n in 2 4; do grep '^{' gpurun_out/rehearse_cornell1080_$n.log | tail -1 > gpurun_out/s10_rehearse_$n.json; done
  timeout -k 10 300 python bench.py --gpus 2 --devices 0,0 --steps 5 --no-cpu-baseline > gpurun_out/s10_inproc.log 2>&1 || { tail -20 gpurun_out/s10_inproc.log; exit 1; }
  grep '^{' gpurun_out/s10_inproc.log | tail -1 > gpurun_out/s10_inproc.json
  for f in gpurun_out/s10_rehearse_2.json gpurun_out/s10_rehearse_4.json gpurun_out/s10_inproc.json; do
  python3 -c "
  import json; d=json.load(open('$f'))
  print('$f', d['n_gpus'], d['value'], d['reduce_backend'], 'fallback', d.get('reduce_fallback'), 'choice_from', d.get('stream_choice_from'))
  for p in d['scaling_breakdown']['per_device']: print('   ', p.get('rank', p.get('device')), p['mode'])"
  done
  timeout -k 10 120 python scripts/probe_step.py --scene cornell --streams 64 --tag units8 > gpurun_out/s10_probe.txt 2>&1 && BDPT_UNITS=8 timeout -k 10 120 python scripts/probe_step.py --scene cornell --streams 64 --tag units8 >> gpurun_out/s10_probe.txt 2>&1; grep '^{' gpurun_out/s10_probe.txt | cut -c1-150
}

s11() {
  ARGS="--scene caustic --streams 128" ROUNDS=2 VARIANTS="pools:BDPT_POOL=16 pools_serial:BDPT_POOL=16;BDPT_FOLD_SERIAL=1 pools_m16:BDPT_POOL=16;BDPT_MAX_LAUNCH_PASSES=16 pools_m8:BDPT_POOL=16;BDPT_MAX_LAUNCH_PASSES=8" OUT=gpurun_out/s11_serial.txt bash scripts/ab.sh || exit 1
  ARGS="--scene cornell --streams 64" ROUNDS=2 VARIANTS="s64: s64_serial:BDPT_FOLD_SERIAL=1" OUT=gpurun_out/s11_serial.txt bash scripts/ab.sh || exit 1
  BDPT_UNITS=8 BDPT_PROF=counts BDPT_JIT_FLAGS=-DBDPT_COUNTS=1 timeout -k 10 150 python scripts/probe_step.py --scene cornell --streams 64 --reps 2 --tag counts_units > gpurun_out/s11_counts_units.txt 2>&1 || exit 1
  BDPT_PROF=counts BDPT_JIT_FLAGS=-DBDPT_COUNTS=1 timeout -k 10 150 python scripts/probe_step.py --scene cornell --streams 64 --reps 2 --tag counts_s64 > gpurun_out/s11_counts_s64.txt 2>&1 || exit 1
  grep -h "bdpt_counts\|^{" gpurun_out/s11_counts_*.txt | cut -c1-200
}

s12() {
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "pool or auto or stream or fold or caustic" > gpurun_out/s12_pytest.log 2>&1 || { tail -30 gpurun_out/s12_pytest.log; exit 1; }
  tail -3 gpurun_out/s12_pytest.log
  MODE=bench ARGS="--workload caustic8 --no-cpu-baseline --steps 20" ROUNDS=2 VARIANTS="serial: concurrent:BDPT_FOLD_SERIAL=0" OUT=gpurun_out/s12_bench.txt bash scripts/ab.sh || exit 1
  timeout -k 10 400 python scripts/shard_probe.py --scene caustic --passes 128 --strong --reps 3 > gpurun_out/s12_caustic_strong.txt 2>&1 || { tail -20 gpurun_out/s12_caustic_strong.txt; exit 1; }
  tail -12 gpurun_out/s12_caustic_strong.txt
}

s13() {
  timeout -k 10 500 python scripts/shard_probe.py --scene caustic --passes 128 --strong --reps 20 > gpurun_out/s13_caustic_strong.txt 2>&1 || { tail -20 gpurun_out/s13_caustic_strong.txt; exit 1; }
  tail -8 gpurun_out/s13_caustic_strong.txt
}

s14() {
  BDPT_UNITS=8 BDPT_PROF=counts BDPT_JIT_FLAGS=-DBDPT_COUNTS=1 timeout -k 10 200 python scripts/probe_step.py --scene cornell --streams 64 --reps 2 --tag counts_units > gpurun_out/s14_counts_units.txt 2>&1 || { tail -20 gpurun_out/s14_counts_units.txt; exit 1; }
  grep -h "bdpt_counts" gpurun_out/s14_counts_units.txt
  timeout -k 10 500 python scripts/shard_probe.py --scene caustic --passes 128 --strong --reps 20 > gpurun_out/s14_caustic_strong.txt 2>&1 || { tail -20 gpurun_out/s14_caustic_strong.txt; exit 1; }
  tail -8 gpurun_out/s14_caustic_strong.txt
}

s16() {
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "pool or auto or stream or fold or caustic or shard" > gpurun_out/s16_pytest.log 2>&1 || { tail -30 gpurun_out/s16_pytest.log; exit 1; }
  tail -2 gpurun_out/s16_pytest.log
  BDPT_FOLD_ROWS=1 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "stream and not pool" > gpurun_out/s16_pytest_rows.log 2>&1 || { tail -30 gpurun_out/s16_pytest_rows.log; exit 1; }
  tail -2 gpurun_out/s16_pytest_rows.log
  MODE=bench ARGS="--workload caustic8 --no-cpu-baseline --steps 20" ROUNDS=2 VARIANTS="rows: tiles:BDPT_FOLD_ROWS=0" OUT=gpurun_out/s16_ab.txt bash scripts/ab.sh || exit 1
  ARGS="--scene cornell --streams 64" ROUNDS=2 VARIANTS="s64: s64rows:BDPT_FOLD_ROWS=1" OUT=gpurun_out/s16_ab.txt bash scripts/ab.sh || exit 1
  MODE=bench ARGS="--workload weak64 --no-cpu-baseline --steps 6" ROUNDS=2 VARIANTS="w64: w64rows:BDPT_FOLD_ROWS=1" OUT=gpurun_out/s16_ab.txt bash scripts/ab.sh || exit 1
}

s17() {
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s17_pytest.log 2>&1 || { tail -30 gpurun_out/s17_pytest.log; exit 1; }
  tail -2 gpurun_out/s17_pytest.log
  timeout -k 10 300 python bench.py --workload caustic8 > gpurun_out/s17_bench_caustic8.json 2> gpurun_out/s17_bench_caustic8.err || exit 1
  tail -1 gpurun_out/s17_bench_caustic8.json | cut -c1-400
  timeout -k 10 400 python bench.py > gpurun_out/s17_bench.json 2> gpurun_out/s17_bench.err || exit 1
  tail -1 gpurun_out/s17_bench.json | cut -c1-400
}

s18() {
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "pool or auto or stream or fold or caustic or shard or config" > gpurun_out/s18_pytest.log 2>&1 || { tail -30 gpurun_out/s18_pytest.log; exit 1; }
  tail -2 gpurun_out/s18_pytest.log
  MODE=bench ARGS="--workload caustic8 --no-cpu-baseline --steps 20" ROUNDS=3 VARIANTS="sparse:" OUT=gpurun_out/s18_ab.txt bash scripts/ab.sh || exit 1
  timeout -k 10 500 python scripts/shard_probe.py --scene caustic --passes 128 --strong --reps 20 --ns 1,8 > gpurun_out/s18_caustic_strong.txt 2>&1 || { tail -20 gpurun_out/s18_caustic_strong.txt; exit 1; }
  tail -4 gpurun_out/s18_caustic_strong.txt
}

s19() {
  for v in "base:" "g16r4:BDPT_POOL_GRID=16;BDPT_POOL=4" "g16r2:BDPT_POOL_GRID=16;BDPT_POOL=2" "g8r2:BDPT_POOL_GRID=8;BDPT_POOL=2" "g64r8:BDPT_POOL_GRID=64;BDPT_POOL=8" "g32r4:BDPT_POOL_GRID=32;BDPT_POOL=4"; do
    tag=${v%%:*}; envs=${v#*:}; IFS=';' read -r -a assign <<< "$envs"
    env "${assign[@]}" timeout -k 10 200 python scripts/shard_probe.py --scene caustic --passes 128 --strong --reps 20 --ns 8 > gpurun_out/s19_$tag.txt 2>&1 || { tail -5 gpurun_out/s19_$tag.txt; exit 1; }
    echo "$tag $(grep '"streams_req": 0' gpurun_out/s19_$tag.txt | tail -1)" | tee -a gpurun_out/s19_grid.txt
  done
}

s20() {
  for r in 1 2 3; do
  for v in "base:" "g16r4:BDPT_POOL_GRID=16;BDPT_POOL=4" "g64r8:BDPT_POOL_GRID=64;BDPT_POOL=8" "g128r16:BDPT_POOL_GRID=128;BDPT_POOL=16" "g64r16:BDPT_POOL_GRID=64;BDPT_POOL=16"; do
    tag=${v%%:*}; envs=${v#*:}; IFS=';' read -r -a assign <<< "$envs"
    env "${assign[@]}" timeout -k 10 200 python scripts/shard_probe.py --scene caustic --passes 128 --strong --reps 30 --ns 8 > gpurun_out/s20_$tag.txt 2>&1 || { tail -5 gpurun_out/s20_$tag.txt; exit 1; }
    echo "$r $tag $(grep '"streams_req": 0' gpurun_out/s20_$tag.txt | tail -1)" | tee -a gpurun_out/s20_grid.txt
  done
  done
}

s21() {
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "pool" > gpurun_out/s21_pytest.log 2>&1 || { tail -30 gpurun_out/s21_pytest.log; exit 1; }
  tail -1 gpurun_out/s21_pytest.log
  timeout -k 10 500 python scripts/shard_probe.py --scene caustic --passes 128 --strong --reps 30 > gpurun_out/s21_caustic_strong.txt 2>&1 || { tail -20 gpurun_out/s21_caustic_strong.txt; exit 1; }
  grep '"streams_req": 0' gpurun_out/s21_caustic_strong.txt
  timeout -k 10 500 python scripts/shard_probe.py --scene caustic --passes 128 --strong --reps 30 > gpurun_out/s21_caustic_strong2.txt 2>&1 || { tail -20 gpurun_out/s21_caustic_strong2.txt; exit 1; }
  grep '"streams_req": 0' gpurun_out/s21_caustic_strong2.txt
}

s22() {
  NS="2 4" WORKLOADS="caustic8 cornell1080" STEPS_N=4 bash scripts/rehearse.sh || exit 1
  NS="2" WORKLOADS="weak64" STEPS_N=2 bash scripts/rehearse.sh || exit 1
  for f in gpurun_out/rehearse_caustic8_2.log gpurun_out/rehearse_caustic8_4.log gpurun_out/rehearse_cornell1080_2.log gpurun_out/rehearse_cornell1080_4.log gpurun_out/rehearse_weak64_2.log; do
  grep '^{' $f | tail -1 | python3 -c "
  import json,sys; d=json.loads(sys.stdin.read())
  sb=d['scaling_breakdown']
  print('$f', d['n_gpus'], d['value'], d['reduce_backend'], 'render', sb['render_s'], 'reduce', sb['reduce_s'])"
  done
}

s23() {
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "pool or auto or stream or fold or caustic or shard or config" > gpurun_out/s23_pytest.log 2>&1 || { tail -30 gpurun_out/s23_pytest.log; exit 1; }
  tail -1 gpurun_out/s23_pytest.log
  MODE=bench ARGS="--workload caustic8 --no-cpu-baseline --steps 20" ROUNDS=3 VARIANTS="bits:" OUT=gpurun_out/s23_ab.txt bash scripts/ab.sh || exit 1
  rm -rf gpurun_out/prof_s23 && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_s23 -o run --output-format csv -- python3 bench.py --workload caustic8 --no-cpu-baseline --steps 10 > gpurun_out/prof_s23.log 2>&1 || exit 1
  head -4 gpurun_out/prof_s23/run_kernel_stats.csv | cut -c1-150
}

s24() {
  BDPT_POOL=16 BDPT_PROF=counts BDPT_JIT_FLAGS=-DBDPT_COUNTS=1 timeout -k 10 200 python scripts/probe_step.py --scene caustic --streams 128 --reps 2 --tag counts_pools > gpurun_out/s24_counts_pools.txt 2>&1 || { tail -20 gpurun_out/s24_counts_pools.txt; exit 1; }
  grep -h "bdpt_counts" gpurun_out/s24_counts_pools.txt
}

s27() {
  MODE=bench ARGS="--workload caustic8 --no-cpu-baseline --steps 20" ROUNDS=3 VARIANTS="u16: u8:BDPT_FOLD_U=8 u32:BDPT_FOLD_U=32" OUT=gpurun_out/s27_fold_u.txt bash scripts/ab.sh || exit 1
}

s28() {
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s28_pytest.log 2>&1 || { tail -30 gpurun_out/s28_pytest.log; exit 1; }
  tail -1 gpurun_out/s28_pytest.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/s28_smoke.log 2>&1 || { tail -20 gpurun_out/s28_smoke.log; exit 1; }
  tail -1 gpurun_out/s28_smoke.log
  timeout -k 10 400 python bench.py > gpurun_out/s28_bench.json 2> gpurun_out/s28_bench.err || exit 1
  timeout -k 10 300 python bench.py --workload caustic8 > gpurun_out/s28_bench_caustic8.json 2> gpurun_out/s28_bench_caustic8.err || exit 1
  timeout -k 10 400 python bench.py --workload weak64 > gpurun_out/s28_bench_weak64.json 2> gpurun_out/s28_bench_weak64.err || exit 1
  for f in s28_bench s28_bench_caustic8 s28_bench_weak64; do tail -1 gpurun_out/$f.json | cut -c1-120; done
}

s29() {
  timeout -k 10 900 python scripts/shard_probe.py --scene cornell --passes 128 --reps 3 > gpurun_out/s29_cornell_weak.txt 2>&1 || { tail -20 gpurun_out/s29_cornell_weak.txt; exit 1; }
  grep '"streams_req": 0' gpurun_out/s29_cornell_weak.txt
  timeout -k 10 900 python scripts/shard_probe.py --workload weak64 --reps 2 > gpurun_out/s29_weak64_bands.txt 2>&1 || { tail -20 gpurun_out/s29_weak64_bands.txt; exit 1; }
  tail -1 gpurun_out/s29_weak64_bands.txt
}

s30() {
  ARGS="--scene synthetic64 --width 4097 --height 513 --streams 64" ROUNDS=2 VARIANTS="s64: units8:BDPT_UNITS=8 units16:BDPT_UNITS=16 pools:BDPT_POOL=16" OUT=gpurun_out/s30_weak64_modes.txt LIMIT=300 bash scripts/ab.sh || exit 1
}

s31() {
  timeout -k 10 300 python -u -m pytest tests/test_gpu_pool.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "pool or auto" > gpurun_out/s31_pytest.log 2>&1 || { tail -30 gpurun_out/s31_pytest.log; exit 1; }
  tail -1 gpurun_out/s31_pytest.log
  MODE=bench ARGS="--workload caustic8 --no-cpu-baseline --steps 20" ROUNDS=2 VARIANTS="skip: noskip:BDPT_JIT_FLAGS=-DBDPT_POOL_NOSKIP=1" OUT=gpurun_out/s31_ab.txt bash scripts/ab.sh || exit 1
  for r in 1 2; do for v in "skip:" "noskip:BDPT_JIT_FLAGS=-DBDPT_POOL_NOSKIP=1"; do
    tag=${v%%:*}; envs=${v#*:}; IFS=';' read -r -a assign <<< "$envs"
    env "${assign[@]}" timeout -k 10 200 python scripts/shard_probe.py --scene caustic --passes 128 --strong --reps 30 --ns 1,8 > gpurun_out/s31_$tag.txt 2>&1 || { tail -5 gpurun_out/s31_$tag.txt; exit 1; }
    echo "$r $tag $(grep '"streams_req": 0' gpurun_out/s31_$tag.txt | tr '\n' ' ')" | tee -a gpurun_out/s31_n8.txt
  done; done
}

s32() {
  for r in 1 2; do for v in "skip:BDPT_POOL=16" "noskip:BDPT_POOL=16;BDPT_JIT_FLAGS=-DBDPT_POOL_NOSKIP=1"; do
    tag=${v%%:*}; envs=${v#*:}; IFS=';' read -r -a assign <<< "$envs"
    env "${assign[@]}" timeout -k 10 200 python scripts/probe_step.py --scene caustic --streams 128 --reps 10 --tag $tag > gpurun_out/s32_n1_$tag.txt 2>&1 || { tail -5 gpurun_out/s32_n1_$tag.txt; exit 1; }
    echo "$r N1 $(grep '^{' gpurun_out/s32_n1_$tag.txt | tail -1 | cut -c1-160)" | tee -a gpurun_out/s32.txt
  done; done
  for r in 1 2; do for v in "skip:BDPT_POOL=4" "noskip:BDPT_POOL=4;BDPT_JIT_FLAGS=-DBDPT_POOL_NOSKIP=1"; do
    tag=${v%%:*}; envs=${v#*:}; IFS=';' read -r -a assign <<< "$envs"
    env "${assign[@]}" timeout -k 10 200 python scripts/shard_probe.py --scene caustic --passes 128 --strong --reps 30 --ns 8 > gpurun_out/s32_n8_$tag.txt 2>&1 || { tail -5 gpurun_out/s32_n8_$tag.txt; exit 1; }
    echo "$r N8 $tag $(grep '"streams_req": 0' gpurun_out/s32_n8_$tag.txt | tail -1)" | tee -a gpurun_out/s32.txt
  done; done
}

s33() {
  timeout -k 10 300 python -u -m pytest tests/test_gpu_pool.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "pool or auto" > gpurun_out/s33_pytest.log 2>&1 || { tail -30 gpurun_out/s33_pytest.log; exit 1; }
  tail -1 gpurun_out/s33_pytest.log
  for r in 1 2; do for v in "early:" "late:BDPT_JIT_FLAGS=-DBDPT_POOL_EARLY=0"; do
    tag=${v%%:*}; envs=${v#*:}; IFS=';' read -r -a assign <<< "$envs"
    env "${assign[@]}" BDPT_POOL=16 timeout -k 10 200 python scripts/probe_step.py --scene caustic --streams 128 --reps 10 --tag $tag > gpurun_out/s33_n1.txt 2>&1 || { tail -5 gpurun_out/s33_n1.txt; exit 1; }
    echo "$r N1 $(grep '^{' gpurun_out/s33_n1.txt | tail -1 | cut -c1-160)" | tee -a gpurun_out/s33.txt
    env "${assign[@]}" BDPT_POOL=4 timeout -k 10 200 python scripts/shard_probe.py --scene caustic --passes 128 --strong --reps 30 --ns 8 > gpurun_out/s33_n8.txt 2>&1 || { tail -5 gpurun_out/s33_n8.txt; exit 1; }
    echo "$r N8 $tag $(grep '"streams_req": 0' gpurun_out/s33_n8.txt | tail -1)" | tee -a gpurun_out/s33.txt
  done; done
}

s34() {
  for P in 32 64 128; do
    BDPT_POOL=4 timeout -k 10 200 python scripts/shard_probe.py --scene caustic --passes $P --strong --reps 30 --ns 1,8 > gpurun_out/s34_p$P.txt 2>&1 || { tail -5 gpurun_out/s34_p$P.txt; exit 1; }
    echo "P=$P $(grep '"streams_req": 0' gpurun_out/s34_p$P.txt | tr '\n' ' ')" | tee -a gpurun_out/s34.txt
  done
}

s35() {
  ARGS="--scene cornell --streams 64" ROUNDS=2 VARIANTS="k48:BDPT_UNITS=8 k32:BDPT_UNITS=8;BDPT_JIT_FLAGS=-DBDPT_REGEN_K=32 k56:BDPT_UNITS=8;BDPT_JIT_FLAGS=-DBDPT_REGEN_K=56 k64:BDPT_UNITS=8;BDPT_JIT_FLAGS=-DBDPT_REGEN_K=64 k16:BDPT_UNITS=8;BDPT_JIT_FLAGS=-DBDPT_REGEN_K=16" OUT=gpurun_out/s35_regen_units.txt bash scripts/ab.sh || exit 1
}

s36() {
  BDPT_POOL_OVERLAP=1 timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "pool or auto or stream or fold or caustic or shard or config or multi or checkpoint or replay" > gpurun_out/s36_pytest_overlap.log 2>&1 || { tail -30 gpurun_out/s36_pytest_overlap.log; exit 1; }
  tail -1 gpurun_out/s36_pytest_overlap.log
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "pool or auto" > gpurun_out/s36_pytest.log 2>&1 || { tail -30 gpurun_out/s36_pytest.log; exit 1; }
  tail -1 gpurun_out/s36_pytest.log
  MODE=bench ARGS="--workload caustic8 --no-cpu-baseline --steps 20" ROUNDS=2 VARIANTS="serial: overlap:BDPT_POOL_OVERLAP=1" OUT=gpurun_out/s36_ab.txt bash scripts/ab.sh || exit 1
  for r in 1 2; do for v in "serial:BDPT_POOL=4" "overlap:BDPT_POOL=4;BDPT_POOL_OVERLAP=1"; do
    tag=${v%%:*}; envs=${v#*:}; IFS=';' read -r -a assign <<< "$envs"
    env "${assign[@]}" timeout -k 10 200 python scripts/shard_probe.py --scene caustic --passes 128 --strong --reps 30 --ns 8 > gpurun_out/s36_n8.txt 2>&1 || { tail -5 gpurun_out/s36_n8.txt; exit 1; }
    echo "$r N8 $tag $(grep '"streams_req": 0' gpurun_out/s36_n8.txt | tail -1)" | tee -a gpurun_out/s36_ab.txt
  done; done
}

s37() {
  BDPT_POOL_OVERLAP=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "pool or auto or caustic or multi or checkpoint" > gpurun_out/s37_pytest_overlap.log 2>&1 || { tail -30 gpurun_out/s37_pytest_overlap.log; exit 1; }
  tail -1 gpurun_out/s37_pytest_overlap.log
  MODE=bench ARGS="--workload caustic8 --no-cpu-baseline --steps 20" ROUNDS=2 VARIANTS="serial: overlap:BDPT_POOL_OVERLAP=1" OUT=gpurun_out/s37_ab.txt bash scripts/ab.sh || exit 1
  for r in 1 2; do for v in "serial:BDPT_POOL=16" "overlap:BDPT_POOL=16;BDPT_POOL_OVERLAP=1"; do
    tag=${v%%:*}; envs=${v#*:}; IFS=';' read -r -a assign <<< "$envs"
    env "${assign[@]}" timeout -k 10 200 python scripts/probe_step.py --scene caustic --streams 128 --reps 20 --tag $tag > gpurun_out/s37_n1.txt 2>&1 || { tail -5 gpurun_out/s37_n1.txt; exit 1; }
    echo "$r N1 $(grep '^{' gpurun_out/s37_n1.txt | tail -1 | cut -c1-140)" | tee -a gpurun_out/s37_ab.txt
  done; done
  for r in 1 2; do for v in "serial:" "overlap:BDPT_POOL_OVERLAP=1"; do
    tag=${v%%:*}; envs=${v#*:}; IFS=';' read -r -a assign <<< "$envs"
    env "${assign[@]}" timeout -k 10 300 python scripts/shard_probe.py --scene caustic --passes 128 --strong --reps 30 > gpurun_out/s37_strong.txt 2>&1 || { tail -5 gpurun_out/s37_strong.txt; exit 1; }
    echo "$r strong $tag $(grep '"streams_req": 0' gpurun_out/s37_strong.txt | cut -c1-120 | tr '\n' ' ')" | tee -a gpurun_out/s37_ab.txt
  done; done
}

s38() {
  for v in "overlap:" "serial:BDPT_POOL_OVERLAP=0"; do
    tag=${v%%:*}; envs=${v#*:}; IFS=';' read -r -a assign <<< "$envs"
    rm -rf gpurun_out/prof_s38_$tag
    env "${assign[@]}" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_s38_$tag -o run --output-format csv -- python3 bench.py --workload caustic8 --no-cpu-baseline --steps 20 > gpurun_out/prof_s38_$tag.log 2>&1 || exit 1
    echo "$tag $(grep '^{' gpurun_out/prof_s38_$tag.log | tail -1 | cut -c1-100)"; head -3 gpurun_out/prof_s38_$tag/run_kernel_stats.csv | cut -c1-120
  done
}

s39() {
  for P in 32 64 128; do
    BDPT_UNITS=8 timeout -k 10 200 python scripts/probe_step.py --scene cornell --passes $P --streams 64 --reps 4 --tag u$P > gpurun_out/s39_u$P.txt 2>&1 || { tail -5 gpurun_out/s39_u$P.txt; exit 1; }
    echo "units P=$P $(grep '^{' gpurun_out/s39_u$P.txt | tail -1 | cut -c1-170)" | tee -a gpurun_out/s39.txt
    timeout -k 10 200 python scripts/probe_step.py --scene cornell --passes $P --streams $((P/2)) --reps 4 --tag s$P > gpurun_out/s39_s$P.txt 2>&1 || { tail -5 gpurun_out/s39_s$P.txt; exit 1; }
    echo "streams P=$P $(grep '^{' gpurun_out/s39_s$P.txt | tail -1 | cut -c1-170)" | tee -a gpurun_out/s39.txt
  done
}

s40() {
  timeout -k 10 600 python -u -m pytest tests/test_gpu_units.py tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > gpurun_out/s40_pytest.log 2>&1 || { tail -30 gpurun_out/s40_pytest.log; exit 1; }
  tail -1 gpurun_out/s40_pytest.log
  ARGS="--scene cornell --streams 64" ROUNDS=3 VARIANTS="taper:BDPT_UNITS=8 flat:BDPT_UNITS=8;BDPT_UNITS_TAPER=0 s64:" OUT=gpurun_out/s40_ab.txt bash scripts/ab.sh || exit 1
}

s41() {
  for U in 4 8 16; do for P in 32 128; do
    BDPT_UNITS=$U timeout -k 10 200 python scripts/probe_step.py --scene cornell --passes $P --streams 64 --reps 4 --tag u${U}p$P > gpurun_out/s41.tmp 2>&1 || { tail -5 gpurun_out/s41.tmp; exit 1; }
    echo "U=$U P=$P $(grep '^{' gpurun_out/s41.tmp | tail -1 | cut -c1-150)" | tee -a gpurun_out/s41.txt
  done; done
}

s42() {
  for v in "table:" "ablate:BDPT_JIT_FLAGS=-DBDPT_SCT_ABLATE=1"; do
    tag=${v%%:*}; envs=${v#*:}; IFS=';' read -r -a assign <<< "$envs"
    rm -rf gpurun_out/pmc_s42_$tag
    env "${assign[@]}" BDPT_UNITS=8 timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/pmc_s42_$tag -o run --output-format csv -- python3 scripts/probe_step.py --scene cornell --streams 64 --reps 2 --tag $tag > gpurun_out/pmc_s42_$tag.log 2>&1 || exit 1
    echo "$tag done"
  done
}

s44() {
  ARGS="--scene caustic --streams 128 --reps 10" ROUNDS=2 VARIANTS="g64r16:BDPT_POOL=16;BDPT_POOL_GRID=64 g32r8:BDPT_POOL=8;BDPT_POOL_GRID=32 g128r32:BDPT_POOL=32;BDPT_POOL_GRID=128 g64r8:BDPT_POOL=8;BDPT_POOL_GRID=64 g64r32:BDPT_POOL=32;BDPT_POOL_GRID=64" OUT=gpurun_out/s44_pool_shape.txt bash scripts/ab.sh || exit 1
}

s45() {
  ARGS="--scene caustic --streams 128 --reps 10" ROUNDS=2 VARIANTS="g128r32:BDPT_POOL=32;BDPT_POOL_GRID=128 g256r64:BDPT_POOL=64;BDPT_POOL_GRID=256 g128r64:BDPT_POOL=64;BDPT_POOL_GRID=128 g256r32:BDPT_POOL=32;BDPT_POOL_GRID=256" OUT=gpurun_out/s45_pool_shape.txt bash scripts/ab.sh || exit 1
  for r in 1 2; do for v in "g16r4:BDPT_POOL=4;BDPT_POOL_GRID=16" "g32r8:BDPT_POOL=8;BDPT_POOL_GRID=32" "g64r16:BDPT_POOL=16;BDPT_POOL_GRID=64"; do
    tag=${v%%:*}; envs=${v#*:}; IFS=';' read -r -a assign <<< "$envs"
    env "${assign[@]}" timeout -k 10 300 python scripts/shard_probe.py --scene caustic --passes 128 --strong --reps 30 --ns 4,8 > gpurun_out/s45_sh.txt 2>&1 || { tail -5 gpurun_out/s45_sh.txt; exit 1; }
    echo "$r $tag $(grep '"streams_req": 0' gpurun_out/s45_sh.txt | cut -c1-75 | tr '\n' ' ')" | tee -a gpurun_out/s45_pool_shape.txt
  done; done
}

s46() {
  for r in 1 2; do for v in "g64r16:BDPT_POOL=16;BDPT_POOL_GRID=64" "g128r32:BDPT_POOL=32;BDPT_POOL_GRID=128" "g128r64:BDPT_POOL=64;BDPT_POOL_GRID=128" "g64r32:BDPT_POOL=32;BDPT_POOL_GRID=64"; do
    tag=${v%%:*}; envs=${v#*:}; IFS=';' read -r -a assign <<< "$envs"
    env "${assign[@]}" timeout -k 10 300 python scripts/shard_probe.py --scene caustic --passes 128 --strong --reps 30 --ns 2,4,8 > gpurun_out/s46_sh.txt 2>&1 || { tail -5 gpurun_out/s46_sh.txt; exit 1; }
    echo "$r $tag $(grep '"streams_req": 0' gpurun_out/s46_sh.txt | cut -c1-75 | tr '\n' ' ')" | tee -a gpurun_out/s46_pool_shape.txt
  done; done
}

s47() {
  timeout -k 10 300 python -u -m pytest tests/test_gpu_pool.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "pool or auto" > gpurun_out/s47_pytest.log 2>&1 || { tail -30 gpurun_out/s47_pytest.log; exit 1; }
  tail -1 gpurun_out/s47_pytest.log
  timeout -k 10 300 python bench.py --workload caustic8 > gpurun_out/s47_bench_caustic8.json 2> gpurun_out/s47_bench_caustic8.err || exit 1
  tail -1 gpurun_out/s47_bench_caustic8.json | cut -c1-120
  timeout -k 10 500 python scripts/shard_probe.py --scene caustic --passes 128 --strong --reps 30 > gpurun_out/s47_strong.txt 2>&1 || { tail -5 gpurun_out/s47_strong.txt; exit 1; }
  grep '"streams_req": 0' gpurun_out/s47_strong.txt | cut -c1-150
}

s48() {
  for r in 1 2; do for v in "g64r16:BDPT_POOL=16;BDPT_POOL_GRID=64" "g64r8:BDPT_POOL=8;BDPT_POOL_GRID=64" "g32r16:BDPT_POOL=16;BDPT_POOL_GRID=32" "g128r16:BDPT_POOL=16;BDPT_POOL_GRID=128" "g32r8:BDPT_POOL=8;BDPT_POOL_GRID=32"; do
    tag=${v%%:*}; envs=${v#*:}; IFS=';' read -r -a assign <<< "$envs"
    env "${assign[@]}" timeout -k 10 300 python scripts/shard_probe.py --scene caustic --passes 128 --strong --reps 30 --ns 8 > gpurun_out/s48_sh.txt 2>&1 || { tail -5 gpurun_out/s48_sh.txt; exit 1; }
    echo "$r $tag $(grep '"streams_req": 0' gpurun_out/s48_sh.txt | cut -c1-75 | tr '\n' ' ')" | tee -a gpurun_out/s48_pool_shape_eighth.txt
  done; done
}

s49() {
  for r in 1 2 3; do for v in "g64r16:BDPT_POOL=16;BDPT_POOL_GRID=64" "g128r16:BDPT_POOL=16;BDPT_POOL_GRID=128" "g128r32:BDPT_POOL=32;BDPT_POOL_GRID=128" "g256r16:BDPT_POOL=16;BDPT_POOL_GRID=256" "g128r8:BDPT_POOL=8;BDPT_POOL_GRID=128" "g256r8:BDPT_POOL=8;BDPT_POOL_GRID=256"; do
    tag=${v%%:*}; envs=${v#*:}; IFS=';' read -r -a assign <<< "$envs"
    env "${assign[@]}" timeout -k 10 300 python scripts/shard_probe.py --scene caustic --passes 128 --strong --reps 30 --ns 8 > gpurun_out/s49_sh.txt 2>&1 || { tail -5 gpurun_out/s49_sh.txt; exit 1; }
    echo "$r $tag $(grep '"streams_req": 0' gpurun_out/s49_sh.txt | cut -c1-75 | tr '\n' ' ')" | tee -a gpurun_out/s49_pool_shape_eighth.txt
  done; done
}

s50() {
  timeout -k 10 300 python -u -m pytest tests/test_gpu_pool.py -x -q --timeout 300 --timeout-method thread > gpurun_out/s50_pytest.log 2>&1 || { tail -30 gpurun_out/s50_pytest.log; exit 1; }
  tail -1 gpurun_out/s50_pytest.log
  for r in 1 2; do for v in "g128r32:BDPT_POOL=32;BDPT_POOL_GRID=128" "g128r16:BDPT_POOL=16;BDPT_POOL_GRID=128"; do
    tag=${v%%:*}; envs=${v#*:}; IFS=';' read -r -a assign <<< "$envs"
    env "${assign[@]}" timeout -k 10 300 python scripts/shard_probe.py --scene caustic --passes 128 --strong --reps 30 --ns 4 > gpurun_out/s50_sh.txt 2>&1 || { tail -5 gpurun_out/s50_sh.txt; exit 1; }
    echo "$r $tag $(grep '"streams_req": 0' gpurun_out/s50_sh.txt | cut -c1-75 | tr '\n' ' ')" | tee -a gpurun_out/s50_pool_shape_quarter.txt
  done; done
  timeout -k 10 500 python scripts/shard_probe.py --scene caustic --passes 128 --strong --reps 30 > gpurun_out/s50_strong.txt 2>&1 || { tail -5 gpurun_out/s50_strong.txt; exit 1; }
  grep '"streams_req": 0' gpurun_out/s50_strong.txt | cut -c1-150
}

s51() {
  timeout -k 10 300 python -u -m pytest tests/test_gpu_pool.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "pool or auto" > gpurun_out/s51_pytest.log 2>&1 || { tail -30 gpurun_out/s51_pytest.log; exit 1; }
  tail -1 gpurun_out/s51_pytest.log
  timeout -k 10 300 python bench.py --workload caustic8 > gpurun_out/s51_bench_caustic8.json 2> gpurun_out/s51_bench_caustic8.err || exit 1
  tail -1 gpurun_out/s51_bench_caustic8.json | cut -c1-120
  timeout -k 10 500 python scripts/shard_probe.py --scene caustic --passes 128 --strong --reps 30 > gpurun_out/s51_strong.txt 2>&1 || { tail -5 gpurun_out/s51_strong.txt; exit 1; }
  grep '"streams_req": 0' gpurun_out/s51_strong.txt | cut -c1-150
}

s52() {
  for r in 1 2; do for v in "g128r32:BDPT_POOL=32;BDPT_POOL_GRID=128" "g256r32:BDPT_POOL=32;BDPT_POOL_GRID=256" "g128r48:BDPT_POOL=48;BDPT_POOL_GRID=128" "g256r16:BDPT_POOL=16;BDPT_POOL_GRID=256" "g128r24:BDPT_POOL=24;BDPT_POOL_GRID=128"; do
    tag=${v%%:*}; envs=${v#*:}; IFS=';' read -r -a assign <<< "$envs"
    env "${assign[@]}" timeout -k 10 300 python scripts/shard_probe.py --scene caustic --passes 128 --strong --reps 30 --ns 2,4 --streams 0 > gpurun_out/s52_sh.txt 2>&1 || { tail -5 gpurun_out/s52_sh.txt; exit 1; }
    echo "$r $tag $(grep '"streams_req": 0' gpurun_out/s52_sh.txt | cut -c1-75 | tr '\n' ' ')" | tee -a gpurun_out/s52_pool_shape_half_quarter.txt
  done; done
}

case "${1:-}" in
  s9|s10|s11|s12|s13|s14|s16|s17|s18|s19|s20|s21|s22|s23|s24|s27|s28|s29|s30|s31|s32|s33|s34|s35|s36|s37|s38|s39|s40|s41|s42|s44|s45|s46|s47|s48|s49|s50|s51|s52) "$1" ;;
  *) echo "usage: $0 {s9|s10|s11|s12|s13|s14|s16|s17|s18|s19|s20|s21|s22|s23|s24|s27|s28|s29|s30|s31|s32|s33|s34|s35|s36|s37|s38|s39|s40|s41|s42|s44|s45|s46|s47|s48|s49|s50|s51|s52}"; exit 2 ;;
esac
