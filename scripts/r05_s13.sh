set -u
cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python scripts/shard_probe.py --scene caustic --passes 128 --strong --reps 20 > gpurun_out/s13_caustic_strong.txt 2>&1 || { tail -20 gpurun_out/s13_caustic_strong.txt; exit 1; }
tail -8 gpurun_out/s13_caustic_strong.txt
