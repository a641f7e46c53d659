#!/bin/bash
# Full GPU suite + smoke + driver bench, then the two-ranks-on-one-GPU RCCL probe
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash benchmarks/gpu_full.sh || exit 1
timeout -k 10 240 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 benchmarks/rccl_two_rank_probe.py > gpurun_out/rccl_two_rank.json 2> gpurun_out/rccl_two_rank.err; echo "probe rc=$?"
cat gpurun_out/rccl_two_rank.json; tail -5 gpurun_out/rccl_two_rank.err
timeout -k 10 300 python3 benchmarks/symeig_timing.py > gpurun_out/symeig_timing_r3.json 2> gpurun_out/symeig_timing.err || { tail -20 gpurun_out/symeig_timing.err; exit 1; }
cat gpurun_out/symeig_timing_r3.json
