#!/bin/bash
# K1 micro kernel vs the general K1 kernel: bench rate and rocprofv3 kernel stats of each.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for MODE in 1 0; do
  export TORCHEVAL_AMD_K1_MICRO=$MODE
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver_m$MODE.json 2> gpurun_out/bench_driver_m$MODE.err || { tail -20 gpurun_out/bench_driver_m$MODE.err; exit 1; }
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 5000 --warmup 500 --no-reference > gpurun_out/bench_5k_m$MODE.json 2>/dev/null || exit 1
  rm -rf /tmp/prof_m$MODE
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_m$MODE -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --gpus 1 --steps 2000 --warmup 200 --no-reference > gpurun_out/prof_m$MODE.log 2>&1 || { tail -20 gpurun_out/prof_m$MODE.log; exit 1; }
  find /tmp/prof_m$MODE -name "*kernel_stats.csv" -exec cp {} gpurun_out/k1_kernel_stats_m$MODE.csv \;
done
for MODE in 1 0; do cat gpurun_out/bench_driver_m$MODE.json gpurun_out/bench_5k_m$MODE.json; head -3 gpurun_out/k1_kernel_stats_m$MODE.csv; done
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/gpu/test_compile_gpu.py tests/gpu/test_torch_ops_gpu.py > gpurun_out/pytest_r3d.log 2>&1; echo "pytest rc=$?"
tail -3 gpurun_out/pytest_r3d.log
