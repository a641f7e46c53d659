#!/bin/bash
# Kernel stats of FID compute at D = 2048 under rocprofv3; the run must exit 0.
#
# rocprofv3 (ROCm 7.0 runtime in torch 2.10) segfaults in process teardown after ANY
# hipLaunchCooperativeKernel, with or without torch: a 30-line HIP program
# (csrc/bench/coop_exit_probe.hip) exits 139 after one cooperative launch and 0 after the same
# launch made with hipLaunchKernel (profiles/exit_bisect_r4/).  K9b's tridiagonalisation is
# our only cooperative launch, so the profiled run selects its plain launch of the same grid
# (TORCHEVAL_AMD_SYMEIG_COOP=0; identical kernel and results, co-resident on an idle GPU, and
# the bounded hand-off spins abort to the library fallback if not).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf /tmp/prof_fid
(cd /tmp && TORCHEVAL_AMD_SYMEIG_COOP=0 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv \
  -d /tmp/prof_fid -o fid -- python3 "$GRAFT_REPO_ROOT/benchmarks/profile_fid_compute.py" \
  > "$GRAFT_REPO_ROOT/gpurun_out/prof_fid.log" 2>&1)
rc=$?
echo "rocprofv3 FID compute profile rc=$rc"
[ $rc -ne 0 ] && { tail -20 gpurun_out/prof_fid.log; exit $rc; }
grep -q "^done" gpurun_out/prof_fid.log || { tail -20 gpurun_out/prof_fid.log; exit 1; }
find /tmp/prof_fid -name "*kernel_stats.csv" -exec cp {} gpurun_out/fid_compute_kernel_stats.csv \;
python3 - <<'PY'
import csv
for r in list(csv.reader(open("gpurun_out/fid_compute_kernel_stats.csv")))[:12]:
    print(r[0][:70], r[1], r[2], r[3])
PY
