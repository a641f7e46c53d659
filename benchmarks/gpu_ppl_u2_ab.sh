#!/bin/bash
# K7 A/B: two-chunk unrolled row body (TORCHEVAL_AMD_PPL_U2=1) vs one chunk per iteration, at
# the default grid cap and at 1024, after the K7 GPU tests with the unrolled body forced on.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TORCHEVAL_AMD_PPL_U2=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/gpu/test_k5_k7_k8.py tests/metrics/text -m gpu > gpurun_out/ppl_u2_tests.log 2>&1 || exit 1
tail -1 gpurun_out/ppl_u2_tests.log
for i in 1 2; do
  for u2 in 0 1; do
    for cap in 0 1024; do
      out=$(TORCHEVAL_AMD_PPL_U2=$u2 TORCHEVAL_AMD_PPL_MAXGRID=$cap timeout -k 10 200 python benchmarks/ppl_ab.py 2>/dev/null) || exit 1
      echo "u2=$u2 cap=$cap $out"
    done
  done
done
