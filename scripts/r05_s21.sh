set -u
cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "pool" > gpurun_out/s21_pytest.log 2>&1 || { tail -30 gpurun_out/s21_pytest.log; exit 1; }
tail -1 gpurun_out/s21_pytest.log
timeout -k 10 500 python scripts/shard_probe.py --scene caustic --passes 128 --strong --reps 30 > gpurun_out/s21_caustic_strong.txt 2>&1 || { tail -20 gpurun_out/s21_caustic_strong.txt; exit 1; }
grep '"streams_req": 0' gpurun_out/s21_caustic_strong.txt
timeout -k 10 500 python scripts/shard_probe.py --scene caustic --passes 128 --strong --reps 30 > gpurun_out/s21_caustic_strong2.txt 2>&1 || { tail -20 gpurun_out/s21_caustic_strong2.txt; exit 1; }
grep '"streams_req": 0' gpurun_out/s21_caustic_strong2.txt
