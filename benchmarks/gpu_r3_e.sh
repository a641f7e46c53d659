#!/bin/bash
# Deferred-fold K1 micro kernel: GPU tests, the driver's bench command, rocprof kernel stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/gpu/test_k1_micro.py tests/gpu/test_k1_classification.py tests/gpu/test_accuracy_gpu.py tests/gpu/test_compile_gpu.py > gpurun_out/pytest_r3e.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_r3e.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver.json 2> gpurun_out/bench_driver.err || { tail -20 gpurun_out/bench_driver.err; exit 1; }
cat gpurun_out/bench_driver.json
timeout -k 10 300 python3 bench.py --gpus 1 --steps 5000 --warmup 500 --no-reference > gpurun_out/bench_5k.json 2>/dev/null || exit 1
cat gpurun_out/bench_5k.json
rm -rf /tmp/prof_e
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_e -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --gpus 1 --steps 20 --warmup 5 > gpurun_out/prof_e.log 2>&1 || { tail -20 gpurun_out/prof_e.log; exit 1; }
find /tmp/prof_e -name "*kernel_stats.csv" -exec cp {} gpurun_out/k1_kernel_stats_driver_cmd_r3.csv \;
cut -c1-160 gpurun_out/k1_kernel_stats_driver_cmd_r3.csv | head -6
