#!/bin/bash
# Counter passes over every pmc_targets workload on the round-5 tree (onesweep K3a passes, K4b,
# K5 v2 at an odd width included): bytes fetched / written per dispatch, SQ instruction mix,
# LDS bank conflicts.  One pass per counter group.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash benchmarks/gpu_pmc_one.sh fetch_r5 FETCH_SIZE > gpurun_out/pmc_fetch_r5.txt 2>&1 || { tail -20 gpurun_out/pmc_fetch_r5.txt; exit 1; }
bash benchmarks/gpu_pmc_one.sh write_r5 WRITE_SIZE > gpurun_out/pmc_write_r5.txt 2>&1 || { tail -20 gpurun_out/pmc_write_r5.txt; exit 1; }
bash benchmarks/gpu_pmc_one.sh sq_r5 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES > gpurun_out/pmc_sq_r5.txt 2>&1 || { tail -20 gpurun_out/pmc_sq_r5.txt; exit 1; }
bash benchmarks/gpu_pmc_one.sh lds_r5 SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_WAVES > gpurun_out/pmc_lds_r5.txt 2>&1 || { tail -20 gpurun_out/pmc_lds_r5.txt; exit 1; }
wc -l gpurun_out/pmc_*_r5.txt
