#!/bin/bash
# Round 4: K1 compare-only kernel (tests, floor, fixed cost, driver bench), sync breakdown
# with the watchdog / group A/B, then the exit-crash bisection under rocprofv3.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/r4g_gpu_tests.log 2>&1
trc=$?; tail -3 gpurun_out/r4g_gpu_tests.log; echo "gpu tests rc=$trc"
[ $trc -gt 1 ] && exit $trc
timeout -k 10 120 ./csrc/bench/k1_floor.bin 8 400 > gpurun_out/k1_floor_r4e.txt 2>&1
rc=$?; cat gpurun_out/k1_floor_r4e.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python benchmarks/sync_breakdown.py > gpurun_out/sync_breakdown_r4c.json 2> gpurun_out/sb.err
rc=$?; cat gpurun_out/sync_breakdown_r4c.json; [ $rc -ne 0 ] && { tail -20 gpurun_out/sb.err; exit $rc; }
timeout -k 10 300 python benchmarks/rccl_sync_floor.py > gpurun_out/sync_floor_r4c.json 2> gpurun_out/sync_floor_r4.err
rc=$?; cat gpurun_out/sync_floor_r4c.json; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python benchmarks/bench_fixed_cost.py > gpurun_out/fc.json 2> gpurun_out/fc.err
rc=$?; echo "fixed cost: $(cat gpurun_out/fc.json)"; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver.json 2> gpurun_out/bench_driver.err
  rc=$?; cat gpurun_out/bench_driver.json; [ $rc -ne 0 ] && exit $rc
done
bash benchmarks/gpu_exit_bisect.sh
exit $trc
