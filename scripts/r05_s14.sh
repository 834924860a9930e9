set -u
cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out; export TMPDIR=/tmp
BDPT_UNITS=8 BDPT_PROF=counts BDPT_JIT_FLAGS=-DBDPT_COUNTS=1 timeout -k 10 200 python scripts/probe_step.py --scene cornell --streams 64 --reps 2 --tag counts_units > gpurun_out/s14_counts_units.txt 2>&1 || { tail -20 gpurun_out/s14_counts_units.txt; exit 1; }
grep -h "bdpt_counts" gpurun_out/s14_counts_units.txt
timeout -k 10 500 python scripts/shard_probe.py --scene caustic --passes 128 --strong --reps 20 > gpurun_out/s14_caustic_strong.txt 2>&1 || { tail -20 gpurun_out/s14_caustic_strong.txt; exit 1; }
tail -8 gpurun_out/s14_caustic_strong.txt
