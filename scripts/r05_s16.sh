set -u
cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "pool or auto or stream or fold or caustic or shard" > gpurun_out/s16_pytest.log 2>&1 || { tail -30 gpurun_out/s16_pytest.log; exit 1; }
tail -2 gpurun_out/s16_pytest.log
BDPT_FOLD_ROWS=1 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "stream and not pool" > gpurun_out/s16_pytest_rows.log 2>&1 || { tail -30 gpurun_out/s16_pytest_rows.log; exit 1; }
tail -2 gpurun_out/s16_pytest_rows.log
MODE=bench ARGS="--workload caustic8 --no-cpu-baseline --steps 20" ROUNDS=2 VARIANTS="rows: tiles:BDPT_FOLD_ROWS=0" OUT=gpurun_out/s16_ab.txt bash scripts/ab.sh || exit 1
ARGS="--scene cornell --streams 64" ROUNDS=2 VARIANTS="s64: s64rows:BDPT_FOLD_ROWS=1" OUT=gpurun_out/s16_ab.txt bash scripts/ab.sh || exit 1
MODE=bench ARGS="--workload weak64 --no-cpu-baseline --steps 6" ROUNDS=2 VARIANTS="w64: w64rows:BDPT_FOLD_ROWS=1" OUT=gpurun_out/s16_ab.txt bash scripts/ab.sh || exit 1
