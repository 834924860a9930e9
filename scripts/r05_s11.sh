set -u
cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out; export TMPDIR=/tmp
ARGS="--scene caustic --streams 128" ROUNDS=2 VARIANTS="pools:BDPT_POOL=16 pools_serial:BDPT_POOL=16;BDPT_FOLD_SERIAL=1 pools_m16:BDPT_POOL=16;BDPT_MAX_LAUNCH_PASSES=16 pools_m8:BDPT_POOL=16;BDPT_MAX_LAUNCH_PASSES=8" OUT=gpurun_out/s11_serial.txt bash scripts/ab.sh || exit 1
ARGS="--scene cornell --streams 64" ROUNDS=2 VARIANTS="s64: s64_serial:BDPT_FOLD_SERIAL=1" OUT=gpurun_out/s11_serial.txt bash scripts/ab.sh || exit 1
BDPT_UNITS=8 BDPT_PROF=counts BDPT_JIT_FLAGS=-DBDPT_COUNTS=1 timeout -k 10 150 python scripts/probe_step.py --scene cornell --streams 64 --reps 2 --tag counts_units > gpurun_out/s11_counts_units.txt 2>&1 || exit 1
BDPT_PROF=counts BDPT_JIT_FLAGS=-DBDPT_COUNTS=1 timeout -k 10 150 python scripts/probe_step.py --scene cornell --streams 64 --reps 2 --tag counts_s64 > gpurun_out/s11_counts_s64.txt 2>&1 || exit 1
grep -h "bdpt_counts\|^{" gpurun_out/s11_counts_*.txt | cut -c1-200
