#!/bin/bash
# Kernel trace of the north-star update stream: per-dispatch duration and start-to-start
# interval of the K1 micro kernel (back-to-back updates), summarised as one JSON line
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf /tmp/k1_trace
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/k1_trace -o k1 -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --gpus 1 --steps 2000 --warmup 50 --no-reference > "$GRAFT_REPO_ROOT/gpurun_out/k1_trace.log" 2>&1) || { tail -20 gpurun_out/k1_trace.log; exit 1; }
f=$(find /tmp/k1_trace -name "*kernel_trace.csv" | head -1)
python3 - "$f" <<'PY'
import csv, json, sys, statistics
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "cls_micro_kernel" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
st = [int(r["Start_Timestamp"]) for r in rows]
en = [int(r["End_Timestamp"]) for r in rows]
dur = [(e - s) / 1e3 for s, e in zip(st, en)]
# the timed run's updates: the last 2000 dispatches, back to back
s2, e2, d2 = st[-2000:], en[-2000:], dur[-2000:]
iv = [(b - a) / 1e3 for a, b in zip(s2, s2[1:])]
gap = [(b - a) / 1e3 for a, b in zip(e2, s2[1:])]
out = {"dispatches": len(rows), "timed_dispatches": len(d2),
       "duration_us": {"median": round(statistics.median(d2), 3), "mean": round(statistics.mean(d2), 3), "min": round(min(d2), 3)},
       "start_to_start_us": {"median": round(statistics.median(iv), 3), "mean": round(statistics.mean(iv), 3)},
       "gap_end_to_next_start_us": {"median": round(statistics.median(gap), 3), "mean": round(statistics.mean(gap), 3)},
       "bytes_per_update": 8192 * 1000 * 4,
       "tb_per_s_at_median_duration": round(8192 * 1000 * 4 / (statistics.median(d2) * 1e-6) / 1e12, 2),
       "tb_per_s_at_median_interval": round(8192 * 1000 * 4 / (statistics.median(iv) * 1e-6) / 1e12, 2)}
print(json.dumps(out))
PY
