#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 200 python3 benchmarks/rccl_direct_primitives.py > gpurun_out/rccl_direct_prims.json 2> gpurun_out/rdp.err || { tail -20 gpurun_out/rdp.err; exit 1; }
cat gpurun_out/rccl_direct_prims.json
