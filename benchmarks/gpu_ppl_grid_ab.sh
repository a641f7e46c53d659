#!/bin/bash
# K7 grid cap A/B: shape-aware default vs forced caps 512 / 1024 (blocks of 4 waves), kernel-only
# timing per shape (benchmarks/ppl_ab.py), after the K7 GPU tests.  Stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/gpu/test_k5_k7_k8.py tests/metrics/text -m gpu > gpurun_out/ppl_grid_tests.log 2>&1 || exit 1
tail -1 gpurun_out/ppl_grid_tests.log
for i in 1 2; do
  for cap in default 512 1024; do
    if [ "$cap" = default ]; then
      out=$(timeout -k 10 200 python benchmarks/ppl_ab.py 2>/dev/null) || exit 1
    else
      out=$(TORCHEVAL_AMD_PPL_MAXGRID=$cap timeout -k 10 200 python benchmarks/ppl_ab.py 2>/dev/null) || exit 1
    fi
    echo "cap=$cap $out"
  done
done
