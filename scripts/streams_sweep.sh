#!/bin/bash
# Pass streams (auto: one pass per lane) vs the fused S = 1 kernel, per scene (bench.py --streams).
#   SCENES="cornell caustic" STREAMS="0 1" bash scripts/streams_sweep.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for sc in ${SCENES:-cornell caustic}; do
  line="$sc"
  for s in ${STREAMS:-0 1}; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --scene $sc --streams $s ${BENCH_ARGS:-} > gpurun_out/sw.log 2>&1 || { echo "STOP $sc $s"; tail -3 gpurun_out/sw.log; exit 1; }
    line="$line  S=$s: $(python -c "import json; d=json.loads(open('gpurun_out/sw.log').read().strip().splitlines()[-1]); print(d['value'], '(', d['config']['pass_streams'], d['config']['traversal'], ')')")"
  done
  echo "$line"
done
