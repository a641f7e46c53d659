#!/bin/bash
# Round-5 evidence on the current tree: kernel census of the whole GPU suite under rocprofv3
# (it is also the suite's pass / fail), smoke(), the driver's bench command, and the driver's
# N=8 launch rehearsed with 8 gloo ranks on the one GPU.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash benchmarks/gpu_r4_suite_kernel_census.sh || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5_smoke.log 2>&1 || { tail -20 gpurun_out/r5_smoke.log; exit 1; }
tail -1 gpurun_out/r5_smoke.log
timeout -k 10 180 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5_final_bench.json 2> gpurun_out/r5_final_bench.err || { tail -20 gpurun_out/r5_final_bench.err; exit 1; }
cat gpurun_out/r5_final_bench.json
BENCH_BACKEND=gloo MASTER_ADDR=127.0.0.1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29631 bench.py --gpus 8 --steps 20 --warmup 5 \
  > gpurun_out/r5_rehearsal_gloo8.log 2>&1
rc=$?; echo "rehearsal8 rc=$rc"; grep '"metric"' gpurun_out/r5_rehearsal_gloo8.log || tail -20 gpurun_out/r5_rehearsal_gloo8.log
exit $rc
