#!/bin/bash
# Rehearse bench.py's multi-rank path on a 1-GPU box: 2 ranks share cuda:0 over gloo
# (the driver's real N > 1 runs use RCCL with one rank per GPU).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
BENCH_BACKEND=gloo MASTER_ADDR=127.0.0.1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 20 --warmup 5 \
  --no-reference > gpurun_out/bench_multi_rehearsal.log 2>&1
rc=$?
grep '"metric"' gpurun_out/bench_multi_rehearsal.log || tail -30 gpurun_out/bench_multi_rehearsal.log
exit $rc
