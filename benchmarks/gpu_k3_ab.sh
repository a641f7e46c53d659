#!/bin/bash
# K3 GPU tests, then kernel stats of multiclass_auroc 100k x 100 and binary_auroc 1M
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/gpu/test_k3_k4_k6.py tests/gpu/test_k3c_curves.py tests/gpu/test_k3m_merge.py > gpurun_out/t_k3.log 2>&1 || { tail -30 gpurun_out/t_k3.log; exit 1; }
tail -1 gpurun_out/t_k3.log
bash benchmarks/gpu_mc_auroc_profile.sh > /dev/null || exit 1
bash benchmarks/gpu_k3_profile.sh > /dev/null || exit 1
python3 - <<'PY'
import csv
for f in ("gpurun_out/mc_auroc_kernel_stats.csv", "gpurun_out/k3_kernel_stats.csv"):
    print("##", f)
    for r in list(csv.reader(open(f)))[1:9]:
        print(r[0][:70], r[1], r[3], r[5], r[6])
PY
