#!/bin/bash
# Run a selection of GPU tests (TESTS="file1 file2 ..." or pytest -k expression in K).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -v -rA --timeout 300 --timeout-method thread ${K:+-k "$K"} > gpurun_out/pytest_sel.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/pytest_sel.log | tail -40; exit $rc
