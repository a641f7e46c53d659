#!/bin/bash
# Round-end checkpoint: the whole GPU suite, smoke(), then the driver's bench command
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_full.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_full.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/pytest_full.log | head -20; exit 1; }
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver.json 2> gpurun_out/bench_driver.err || { tail -20 gpurun_out/bench_driver.err; exit 1; }
cat gpurun_out/bench_driver.json
