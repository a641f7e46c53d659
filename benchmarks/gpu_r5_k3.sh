#!/bin/bash
# Round 5: K3a onesweep sort - GPU tests, A/B against the legacy sort, kernel trace at 1M
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/gpu/test_k3_onesweep.py \
  tests/gpu/test_k3_k4_k6.py tests/gpu/test_k3c_curves.py tests/gpu/test_k3m_merge.py > gpurun_out/r5_k3_tests.log 2>&1 \
  || { tail -40 gpurun_out/r5_k3_tests.log; exit 1; }
tail -1 gpurun_out/r5_k3_tests.log
timeout -k 10 300 python3 -u benchmarks/k3_onesweep_ab.py > gpurun_out/r5_k3_ab.jsonl 2>&1 || { tail -20 gpurun_out/r5_k3_ab.jsonl; exit 1; }
cat gpurun_out/r5_k3_ab.jsonl
bash benchmarks/gpu_k3_profile.sh > /dev/null || exit 1
python3 - <<'PY'
import csv
rows = list(csv.reader(open("gpurun_out/k3_kernel_stats.csv")))
for r in rows[1:12]:
    print(r[0][:90], r[1], r[3])
PY
