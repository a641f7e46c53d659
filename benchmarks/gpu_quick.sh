#!/bin/bash
# quick loop: gpu tests + k1 microbench + bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python benchmarks/bench_k1.py > gpurun_out/bench_k1.json 2> gpurun_out/bench_k1.err &&
timeout -k 10 300 python bench.py --steps 20000 --warmup 1000 > gpurun_out/bench.json 2> gpurun_out/bench.err
echo "exit=$?"
