#!/bin/bash
# K3 / sort GPU tests, then the 1M AUROC/AUPRC kernel profile
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/gpu -k "auroc or auprc or curve or sort or k3 or merge or retrieval" > gpurun_out/t_k3.log 2>&1 || { tail -30 gpurun_out/t_k3.log; exit 1; }
tail -2 gpurun_out/t_k3.log
bash benchmarks/gpu_k3_profile.sh > gpurun_out/k3_prof_out.txt 2>&1 || { tail -20 gpurun_out/k3_prof_out.txt; exit 1; }
python3 - <<'PY'
import csv
rows=list(csv.DictReader(open('gpurun_out/k3_kernel_trace.csv')))
rows.sort(key=lambda r:int(r['Start_Timestamp']))
tail=rows[-14:]
tot=0
for r in tail:
    d=(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1000; tot+=d
    print(f"{r['Kernel_Name'][30:80]:50s} {d:7.2f}")
print('sum', round(tot, 2))
PY
