#!/bin/bash
# Round 5 evidence: bench.py (driver command x3), the full bench suite, FETCH_SIZE of K5 / K5b / K1
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
: > gpurun_out/r5_bench.jsonl
for i in 1 2 3; do
  timeout -k 10 180 python3 bench.py --gpus 1 --steps 20 --warmup 5 >> gpurun_out/r5_bench.jsonl 2> gpurun_out/r5_bench.err || { tail -20 gpurun_out/r5_bench.err; exit 1; }
done
cat gpurun_out/r5_bench.jsonl
timeout -k 10 900 python3 -u benchmarks/bench_suite.py --out gpurun_out/bench_suite_r5.json > gpurun_out/bench_suite_r5.log 2>&1 || { tail -20 gpurun_out/bench_suite_r5.log; exit 1; }
tail -3 gpurun_out/bench_suite_r5.log
export TMPDIR=/tmp
rm -rf /tmp/k5_pmc
(cd /tmp && timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d /tmp/k5_pmc -o k5 \
  -- python3 "$GRAFT_REPO_ROOT/benchmarks/k5_fetch_probe.py" > "$GRAFT_REPO_ROOT/gpurun_out/k5_pmc.log" 2>&1) || { tail -20 gpurun_out/k5_pmc.log; exit 1; }
f=$(find /tmp/k5_pmc -name "*counter_collection.csv" | head -1)
cp "$f" gpurun_out/k5_pmc_counters.csv
python3 - <<'PY'
import csv, json, collections
rows = list(csv.DictReader(open("gpurun_out/k5_pmc_counters.csv")))
rows.sort(key=lambda r: int(r["Dispatch_Id"]))
by = collections.OrderedDict()
for r in rows:
    k = r["Kernel_Name"].split("(")[0][:90]
    by.setdefault(k, []).append(float(r["Counter_Value"]))
out = {"what": "FETCH_SIZE (KB) per dispatch, in dispatch order, per kernel name (benchmarks/k5_fetch_probe.py)", "kernels": by}
json.dump(out, open("gpurun_out/k5_pmc_fetch.json", "w"), indent=1)
for k, v in by.items():
    print(k, len(v), [round(x) for x in v[:10]])
PY
