#!/bin/bash
# K9b workgroup size A/B: 256 threads (default) vs 512 / 1024 (TORCHEVAL_AMD_SYMEIG_NT)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for nt in 512 1024; do
  TORCHEVAL_AMD_SYMEIG_NT=$nt timeout -k 10 240 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/gpu/test_k9b_symeig.py > gpurun_out/r5_k9nt_tests_$nt.log 2>&1 || { tail -30 gpurun_out/r5_k9nt_tests_$nt.log; exit 1; }
  echo "nt $nt tests: $(tail -1 gpurun_out/r5_k9nt_tests_$nt.log)"
done
for nt in 1024 512 256 1024 512 256; do
  TORCHEVAL_AMD_SYMEIG_NT=$nt timeout -k 10 240 python3 benchmarks/symeig_timing.py > gpurun_out/symeig_nt_$nt.json 2> gpurun_out/symeig_nt.err || { tail -20 gpurun_out/symeig_nt.err; exit 1; }
  cp gpurun_out/symeig_nt_$nt.json gpurun_out/symeig_nt_${nt}_$(date +%s).json
  python3 -c "import json; d=json.load(open('gpurun_out/symeig_nt_$nt.json')); print('nt $nt', 'eig512', d['eig_d512']['k9b_ms_min_med'][1], 'eig1000', d['eig_d1000']['k9b_ms_min_med'][1], 'eig2048', d['eig_d2048']['k9b_ms_min_med'][1], 'err2048', d['eig_d2048']['max_abs_err_rel'], 'fid', d['fid_compute_d2048_ms_min_med'][1])"
done
