#!/bin/bash
# round 6 closing session: every gpu-marked test, the BASELINE-table suite, bench.py
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 150 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r6_pytest_gpu.log 2>&1
rc=$?
tail -15 gpurun_out/r6_pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u benchmarks/bench_suite.py --out gpurun_out/r6_bench_suite.json > gpurun_out/r6_bench_suite.log 2>&1 || { tail -20 gpurun_out/r6_bench_suite.log; exit 1; }
tail -45 gpurun_out/r6_bench_suite.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6_smoke.log 2>&1 || { tail -20 gpurun_out/r6_smoke.log; exit 1; }
echo smoke ok
timeout -k 10 300 python -u bench.py > gpurun_out/r6_bench.log 2>&1 || { tail -20 gpurun_out/r6_bench.log; exit 1; }
tail -1 gpurun_out/r6_bench.log
