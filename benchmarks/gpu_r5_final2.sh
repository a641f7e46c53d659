#!/bin/bash
# Round-5 closing evidence on the final tree: the driver's `pytest tests -m gpu`, the kernel
# census of tests/gpu under rocprofv3, smoke(), the driver's bench command twice, the BASELINE
# suite, and the N=8 launch rehearsed with 8 gloo ranks on the one GPU.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r5_gpu_suite_final.log 2>&1 || { tail -30 gpurun_out/r5_gpu_suite_final.log; exit 1; }
echo "gpu suite: $(tail -1 gpurun_out/r5_gpu_suite_final.log)"
bash benchmarks/gpu_r4_suite_kernel_census.sh || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5_smoke.log 2>&1 || { tail -20 gpurun_out/r5_smoke.log; exit 1; }
tail -1 gpurun_out/r5_smoke.log
for i in 1 2; do
  timeout -k 10 180 python3 bench.py > gpurun_out/r5_final_bench_$i.json 2> gpurun_out/r5_final_bench_$i.err || { tail -20 gpurun_out/r5_final_bench_$i.err; exit 1; }
  cat gpurun_out/r5_final_bench_$i.json
done
timeout -k 10 900 python3 -u benchmarks/bench_suite.py --out gpurun_out/bench_suite_r5_final.json > gpurun_out/bench_suite_r5_final.log 2>&1 || { tail -20 gpurun_out/bench_suite_r5_final.log; exit 1; }
tail -2 gpurun_out/bench_suite_r5_final.log
BENCH_BACKEND=gloo MASTER_ADDR=127.0.0.1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29631 bench.py --gpus 8 --steps 20 --warmup 5 \
  > gpurun_out/r5_rehearsal_gloo8_final.log 2>&1
rc=$?; echo "rehearsal8 rc=$rc"; grep '"metric"' gpurun_out/r5_rehearsal_gloo8_final.log || tail -20 gpurun_out/r5_rehearsal_gloo8_final.log
exit $rc
