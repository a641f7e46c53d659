#!/bin/bash
# End-of-session evidence on the final tree: the BASELINE suite, then the 8-rank gloo-on-one-GPU
# rehearsal of the driver's N=8 launch (extras on).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python3 -u benchmarks/bench_suite.py --out gpurun_out/bench_suite_r4b.json > gpurun_out/bench_suite_r4b.log 2>&1
rc=$?; tail -44 gpurun_out/bench_suite_r4b.log; [ $rc -ne 0 ] && exit $rc
BENCH_BACKEND=gloo MASTER_ADDR=127.0.0.1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29631 bench.py --gpus 8 --steps 20 --warmup 5 \
  > gpurun_out/bench_rehearsal_gloo8_final.log 2>&1
rc=$?; echo "rehearsal8 rc=$rc"; grep '"metric"' gpurun_out/bench_rehearsal_gloo8_final.log || tail -20 gpurun_out/bench_rehearsal_gloo8_final.log
exit $rc
