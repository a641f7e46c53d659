#!/bin/bash
# Round 4: lean-kernarg K1 micro kernel - correctness, floor harness, fixed cost, driver bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/gpu/test_k1_micro.py tests/gpu/test_k1_classification.py tests/gpu/test_accuracy_gpu.py > gpurun_out/r4c_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r4c_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 ./csrc/bench/k1_floor.bin 8 400 > gpurun_out/k1_floor_r4b.txt 2>&1
rc=$?; cat gpurun_out/k1_floor_r4b.txt; [ $rc -ne 0 ] && exit $rc
for knob in "" "HIP_FORCE_DEV_KERNARG=1"; do
  env $knob timeout -k 10 200 python benchmarks/bench_fixed_cost.py > gpurun_out/fc.json 2> gpurun_out/fc.err
  rc=$?; echo "fixed cost [$knob]: $(cat gpurun_out/fc.json)"; [ $rc -ne 0 ] && { tail -5 gpurun_out/fc.err; exit $rc; }
done
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver.json 2> gpurun_out/bench_driver.err
  rc=$?; cat gpurun_out/bench_driver.json; [ $rc -ne 0 ] && { tail -5 gpurun_out/bench_driver.err; exit $rc; }
done
