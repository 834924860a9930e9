set -u
cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out; export TMPDIR=/tmp
BDPT_POOL=16 BDPT_PROF=counts BDPT_JIT_FLAGS=-DBDPT_COUNTS=1 timeout -k 10 200 python scripts/probe_step.py --scene caustic --streams 128 --reps 2 --tag counts_pools > gpurun_out/s24_counts_pools.txt 2>&1 || { tail -20 gpurun_out/s24_counts_pools.txt; exit 1; }
grep -h "bdpt_counts" gpurun_out/s24_counts_pools.txt
