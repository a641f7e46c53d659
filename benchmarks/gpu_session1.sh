#!/bin/bash
# GPU session: tests, micro-bench, bench.py, rocprofv3 kernel stats. Every GPU step bounded.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -c "import torch; print(torch.cuda.get_device_name(0))" > gpurun_out/dev.log 2>&1 &&
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python benchmarks/bench_k1.py > gpurun_out/bench_k1.json 2> gpurun_out/bench_k1.err &&
timeout -k 10 300 python bench.py --steps 20000 --warmup 1000 > gpurun_out/bench.json 2> gpurun_out/bench.err &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_bench" -o bench -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 2000 --warmup 100 --no-reference > "$GRAFT_REPO_ROOT/gpurun_out/prof_bench.log" 2>&1
echo "exit=$?"
