#!/bin/bash
# K9b multisection lanes per eigenvalue A/B (TORCHEVAL_AMD_SYMEIG_L)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TORCHEVAL_AMD_SYMEIG_L=32 timeout -k 10 240 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/gpu/test_k9b_symeig.py > gpurun_out/r5_k9L_tests.log 2>&1 || { tail -30 gpurun_out/r5_k9L_tests.log; exit 1; }
echo "L32 tests: $(tail -1 gpurun_out/r5_k9L_tests.log)"
for l in 32 16 64 32 16; do
  TORCHEVAL_AMD_SYMEIG_L=$l timeout -k 10 240 python3 benchmarks/symeig_timing.py > gpurun_out/symeig_L_$l.json 2> gpurun_out/symeig_L.err || { tail -20 gpurun_out/symeig_L.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/symeig_L_$l.json')); print('L $l', 'eig512', d['eig_d512']['k9b_ms_min_med'][1], 'eig1000', d['eig_d1000']['k9b_ms_min_med'][1], 'eig2048', d['eig_d2048']['k9b_ms_min_med'][1], 'err', d['eig_d2048']['max_abs_err_rel'])"
done
