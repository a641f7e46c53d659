#!/bin/bash
# Round 4, first box: the ws > 1 sync kernels (synthetic gathered rows + gloo ranks on cuda:0),
# the direct-RCCL tests, the 8-rank gloo rehearsal of bench.py, and the driver's bench command.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/gpu/test_sync_multirank_kernels.py tests/gpu/test_rccl_direct.py > gpurun_out/r4a_tests.log 2>&1
rc=$?; tail -25 gpurun_out/r4a_tests.log; [ $rc -ne 0 ] && exit $rc
BENCH_BACKEND=gloo MASTER_ADDR=127.0.0.1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29613 bench.py --gpus 8 --steps 20 --warmup 5 \
  > gpurun_out/bench_rehearsal_gloo8_gpu.log 2>&1
rc=$?; echo "rehearsal8 rc=$rc"; grep '"metric"' gpurun_out/bench_rehearsal_gloo8_gpu.log || tail -30 gpurun_out/bench_rehearsal_gloo8_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver.json 2> gpurun_out/bench_driver.err
rc=$?; cat gpurun_out/bench_driver.json; exit $rc
