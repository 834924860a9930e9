#!/bin/bash
# Multi-rank rehearsal on one GPU (bench.py --rehearse: gloo, ranks share the device):
#   NS="2 4" WORKLOADS="cornell1080 caustic8" bash scripts/rehearse.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
port=29611
for w in ${WORKLOADS:-cornell1080}; do
  for n in ${NS:-2 4}; do
    port=$((port+1))
    timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
        --master-port $port bench.py --gpus $n --steps ${STEPS_N:-5} --warmup 3 --no-cpu-baseline --rehearse \
        --workload $w > gpurun_out/rehearse_${w}_$n.log 2>&1 || { echo "STOP $w N=$n"; tail -20 gpurun_out/rehearse_${w}_$n.log; exit 1; }
    echo "$w N=$n: $(grep '^{' gpurun_out/rehearse_${w}_$n.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['unit'], 'n_gpus', d['n_gpus'], 'streams', d['config']['pass_streams'])")"
  done
done
