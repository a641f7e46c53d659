#!/bin/bash
# Counter passes over every pmc_targets workload on the final tree: bytes fetched / written per
# dispatch, and SQ instruction mix.  One pass per counter group (no multi-pass splitting).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash benchmarks/gpu_pmc_one.sh fetch_r4 FETCH_SIZE > gpurun_out/pmc_fetch_r4.txt 2>&1 || { tail -20 gpurun_out/pmc_fetch_r4.txt; exit 1; }
bash benchmarks/gpu_pmc_one.sh write_r4 WRITE_SIZE > gpurun_out/pmc_write_r4.txt 2>&1 || { tail -20 gpurun_out/pmc_write_r4.txt; exit 1; }
bash benchmarks/gpu_pmc_one.sh sq_r4 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES > gpurun_out/pmc_sq_r4.txt 2>&1 || { tail -20 gpurun_out/pmc_sq_r4.txt; exit 1; }
wc -l gpurun_out/pmc_*_r4.txt
