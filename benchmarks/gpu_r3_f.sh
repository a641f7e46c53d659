#!/bin/bash
# Sync breakdown + floors, and PMC passes of the driver bench command (K1 micro kernel).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python3 benchmarks/sync_breakdown.py > gpurun_out/sync_breakdown.json 2> gpurun_out/sync_breakdown.err || { tail -20 gpurun_out/sync_breakdown.err; exit 1; }
cat gpurun_out/sync_breakdown.json
timeout -k 10 200 python3 benchmarks/rccl_sync_floor.py --out gpurun_out/sync_floor.json > /dev/null 2> gpurun_out/sync_floor.err || { tail -20 gpurun_out/sync_floor.err; exit 1; }
cat gpurun_out/sync_floor.json
rm -rf /tmp/pmc_fetch /tmp/pmc_sq
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d /tmp/pmc_fetch -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --gpus 1 --steps 20 --warmup 5 --no-reference > gpurun_out/pmc_fetch.log 2>&1 || { tail -20 gpurun_out/pmc_fetch.log; exit 1; }
find /tmp/pmc_fetch -name "*counter_collection.csv" -exec cp {} gpurun_out/pmc_fetch_r3.csv \;
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU --kernel-trace --output-format csv -d /tmp/pmc_sq -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --gpus 1 --steps 20 --warmup 5 --no-reference > gpurun_out/pmc_sq.log 2>&1 || { tail -20 gpurun_out/pmc_sq.log; exit 1; }
find /tmp/pmc_sq -name "*counter_collection.csv" -exec cp {} gpurun_out/pmc_sq_r3.csv \;
ls -la gpurun_out/pmc_*_r3.csv
