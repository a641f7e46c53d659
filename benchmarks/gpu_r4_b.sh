#!/bin/bash
# Round 4: direct-RCCL plan / timeout / watchdog tests, sync kernels, graphs; the 8-rank gloo
# rehearsal; the sync floor; the K1 floor harness and bench.py's fixed cost under runtime knobs.
# A plain test failure (rc 1) does not stop the measurements; a crash / timeout does.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/gpu/test_rccl_direct.py tests/gpu/test_sync_multirank_kernels.py tests/gpu/test_k1_micro.py \
  tests/gpu/test_accuracy_gpu.py > gpurun_out/r4b_tests.log 2>&1
trc=$?; tail -30 gpurun_out/r4b_tests.log; echo "tests rc=$trc"
[ $trc -gt 1 ] && exit $trc
BENCH_BACKEND=gloo MASTER_ADDR=127.0.0.1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29613 bench.py --gpus 8 --steps 20 --warmup 5 \
  > gpurun_out/bench_rehearsal_gloo8_gpu.log 2>&1
rc=$?; echo "rehearsal8 rc=$rc"; grep '"metric"' gpurun_out/bench_rehearsal_gloo8_gpu.log || tail -30 gpurun_out/bench_rehearsal_gloo8_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python benchmarks/rccl_sync_floor.py > gpurun_out/sync_floor_r4.json 2> gpurun_out/sync_floor_r4.err
rc=$?; cat gpurun_out/sync_floor_r4.json; tail -3 gpurun_out/sync_floor_r4.err; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 ./csrc/bench/k1_floor.bin 8 400 > gpurun_out/k1_floor_r4.txt 2>&1
rc=$?; cat gpurun_out/k1_floor_r4.txt; [ $rc -ne 0 ] && exit $rc
for knob in "" "HIP_FORCE_DEV_KERNARG=1" "HIP_FORCE_DEV_KERNARG=0" "ROC_ACTIVE_WAIT_TIMEOUT=500"; do
  env $knob timeout -k 10 200 python benchmarks/bench_fixed_cost.py > gpurun_out/fc.json 2> gpurun_out/fc.err
  rc=$?; echo "fixed cost [$knob]: $(cat gpurun_out/fc.json)"; [ $rc -ne 0 ] && { tail -5 gpurun_out/fc.err; exit $rc; }
done
exit $trc
