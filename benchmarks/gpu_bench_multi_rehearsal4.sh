#!/bin/bash
# Rehearse bench.py's multi-rank path with 4 ranks sharing cuda:0 over gloo (the driver's real
# N > 1 runs use RCCL with one rank per GPU; RCCL refuses two ranks on one device).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
BENCH_BACKEND=gloo MASTER_ADDR=127.0.0.1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29613 bench.py --gpus 4 --steps 20 --warmup 5 \
  --no-reference > gpurun_out/bench_multi_rehearsal4.log 2>&1
rc=$?
grep '"metric"' gpurun_out/bench_multi_rehearsal4.log || tail -30 gpurun_out/bench_multi_rehearsal4.log
exit $rc
