#!/bin/bash
# K1 micro kernel workgroup size A/B (4 vs 8 waves per workgroup, one wave per row either way):
# numerics, the floor harness and the driver command, interleaved in separate processes.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TORCHEVAL_AMD_K1_WPB=8 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/gpu/test_k1_micro.py tests/gpu/test_accuracy_gpu.py > gpurun_out/wpb_tests.log 2>&1 || { tail -20 gpurun_out/wpb_tests.log; exit 1; }
tail -1 gpurun_out/wpb_tests.log
v() { python3 -c "import json,sys; print(json.loads(sys.stdin.read())['value'])"; }
for i in 1 2 3 4 5 6; do
  for w in 4 8; do
    p=$(TORCHEVAL_AMD_K1_WPB=$w timeout -k 10 60 ./csrc/bench/k1_floor.bin 8 300 2>&1 | grep '"prod (' | sed 's/.*us_per_launch": \([0-9.]*\).*/\1/')
    b=$(TORCHEVAL_AMD_K1_WPB=$w timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 2>/dev/null | v)
    echo "wpb=$w prod_us=$p bench=$b"
  done
done
