#!/bin/bash
# K8 small-D split sweep (kMode 2) against the GEMM.
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u benchmarks/k8_sweep.py --d 512 768 1024 --k 1000 --modes x3 --splits 0 1 2 3 4 6 8 12 --out gpurun_out/k8_smalld.json > gpurun_out/k8_smalld.log 2>&1
python3 -c "
import json
for r in json.load(open('gpurun_out/k8_smalld.json')): print(r['D'], r['K'], r['split'], r['k8_us'], r['gemm_us'], r['speedup_vs_gemm'])
"
