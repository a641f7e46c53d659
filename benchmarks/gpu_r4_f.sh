#!/bin/bash
# Round 4: the whole GPU suite + smoke, then the measurements (K1 floor variants, sync
# breakdown + floors, latency anatomy, fixed cost, driver bench x2) and the FID compute profile
# under rocprofv3 with a torch-only control.  A plain test failure (rc 1) does not stop the
# measurements; a crash / timeout does.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/r4f_gpu_tests.log 2>&1
trc=$?; tail -4 gpurun_out/r4f_gpu_tests.log; echo "gpu tests rc=$trc"
[ $trc -gt 1 ] && exit $trc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -2 gpurun_out/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 ./csrc/bench/k1_floor.bin 8 400 > gpurun_out/k1_floor_r4c.txt 2>&1
rc=$?; cat gpurun_out/k1_floor_r4c.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python benchmarks/sync_breakdown.py > gpurun_out/sync_breakdown_r4.json 2> gpurun_out/sb.err
rc=$?; cat gpurun_out/sync_breakdown_r4.json; [ $rc -ne 0 ] && { tail -20 gpurun_out/sb.err; exit $rc; }
timeout -k 10 300 python benchmarks/rccl_sync_floor.py > gpurun_out/sync_floor_r4.json 2> gpurun_out/sync_floor_r4.err
rc=$?; cat gpurun_out/sync_floor_r4.json; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python benchmarks/latency_anatomy.py > gpurun_out/latency_anatomy_r4.json 2> gpurun_out/la.err
rc=$?; echo "latency anatomy: $(cat gpurun_out/latency_anatomy_r4.json)"; [ $rc -ne 0 ] && { tail -5 gpurun_out/la.err; exit $rc; }
timeout -k 10 200 python benchmarks/bench_fixed_cost.py > gpurun_out/fc.json 2> gpurun_out/fc.err
rc=$?; echo "fixed cost: $(cat gpurun_out/fc.json)"; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver.json 2> gpurun_out/bench_driver.err
  rc=$?; cat gpurun_out/bench_driver.json; [ $rc -ne 0 ] && exit $rc
done
export TMPDIR=/tmp
rm -rf /tmp/prof_fid /tmp/prof_ctl
(cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_fid -o fid -- \
  python3 "$GRAFT_REPO_ROOT/benchmarks/profile_fid_compute.py" > "$GRAFT_REPO_ROOT/gpurun_out/prof_fid.log" 2>&1)
echo "fid profile rc=$?"
find /tmp/prof_fid -name "*kernel_stats.csv" -exec cp {} gpurun_out/fid_compute_kernel_stats_r4.csv \;
(cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_ctl -o ctl -- \
  python3 -c "import torch; x=torch.randn(2048,2048,device='cuda',dtype=torch.float64); y=(x@x).sum().item(); print('done')" \
  > "$GRAFT_REPO_ROOT/gpurun_out/prof_ctl.log" 2>&1)
echo "control (torch only) profile rc=$?"
tail -3 gpurun_out/prof_fid.log gpurun_out/prof_ctl.log
exit $trc
