#!/bin/bash
# round 6, call A: graph-replay fold fix + the 8-rank gloo rehearsal of the N>1
# diagnostics on one GPU + smoke
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/gpu/test_k5_pending.py \
  tests/gpu/test_accuracy_gpu.py tests/gpu/test_k1_micro.py > gpurun_out/r6a_pytest.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6a_smoke.log 2>&1 &&
BENCH_BACKEND=gloo BENCH_EXTRAS=sync timeout -k 10 600 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 8 --steps 20 --warmup 5 \
  --no-reference > gpurun_out/r6a_rehearsal8.log 2>&1
rc=$?
tail -3 gpurun_out/r6a_pytest.log; grep '"metric"' gpurun_out/r6a_rehearsal8.log || tail -30 gpurun_out/r6a_rehearsal8.log
exit $rc
