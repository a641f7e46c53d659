#!/bin/bash
# K7 row-block perplexity: GPU numerics, then the A/B against the wave-per-row kernel.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/gpu/test_k5_k7_k8.py -k k7 > gpurun_out/ppl_tests.log 2>&1
rc=$?; tail -5 gpurun_out/ppl_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python benchmarks/ppl_ab.py > gpurun_out/ppl_rowblock.json && \
TORCHEVAL_AMD_PPL_ROWBLOCK=0 timeout -k 10 200 python benchmarks/ppl_ab.py > gpurun_out/ppl_wave.json
rc=$?; echo "rowblock: $(cat gpurun_out/ppl_rowblock.json)"; echo "wave: $(cat gpurun_out/ppl_wave.json)"; exit $rc
