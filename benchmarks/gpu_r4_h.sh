#!/bin/bash
# Round 4 evidence: rocprofv3 kernel stats of the driver's exact bench command, the FID compute
# profile (must exit 0), the BASELINE suite refresh, and PMC passes over the K1 floor harness.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf /tmp/prof_drv
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_drv -o drv -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --gpus 1 --steps 20 --warmup 5 > "$GRAFT_REPO_ROOT/gpurun_out/prof_drv.log" 2>&1)
rc=$?; echo "driver bench under rocprofv3 rc=$rc"; grep '"metric"' gpurun_out/prof_drv.log | cut -c1-200
[ $rc -ne 0 ] && { tail -10 gpurun_out/prof_drv.log; exit $rc; }
find /tmp/prof_drv -name "*kernel_stats.csv" -exec cp {} gpurun_out/drv_kernel_stats_r4.csv \;
bash benchmarks/gpu_fid_compute_profile.sh || exit $?
cp gpurun_out/fid_compute_kernel_stats.csv gpurun_out/fid_compute_kernel_stats_r4b.csv
timeout -k 10 600 python benchmarks/bench_suite.py --out gpurun_out/bench_suite_r4.json > gpurun_out/bench_suite_r4.log 2>&1
rc=$?; tail -45 gpurun_out/bench_suite_r4.log; [ $rc -ne 0 ] && exit $rc
bash benchmarks/gpu_pmc_k1_floor.sh
