#!/bin/bash
# K7 HBM bytes per launch: one rocprofv3 FETCH_SIZE pass over benchmarks/ppl_ab.py with 1 + 3
# launches per shape, FETCH_SIZE (KB) per perplexity_kernel dispatch vs the logits bytes.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf /tmp/k7_pmc
(cd /tmp && PPL_AB_REPS=3 timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d /tmp/k7_pmc -o k7 \
  -- python3 "$GRAFT_REPO_ROOT/benchmarks/ppl_ab.py" > "$GRAFT_REPO_ROOT/gpurun_out/k7_pmc.log" 2>&1) || exit 1
f=$(find /tmp/k7_pmc -name "*counter_collection.csv" | head -1)
cp "$f" gpurun_out/k7_pmc_counters.csv
python3 - <<'PY'
import csv, json
rows = [r for r in csv.DictReader(open("gpurun_out/k7_pmc_counters.csv")) if "perplexity_kernel" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Dispatch_Id"]))
shapes = [(4096, 32000, 4), (4096, 32000, 2), (16384, 32000, 2), (2048, 128256, 2), (4096, 50257, 4), (65536, 4096, 4), (8192, 1024, 4)]
out = {"what": "K7 FETCH_SIZE per perplexity_kernel dispatch (KB, median of the 3 timed launches) vs logits bytes", "n_dispatches": len(rows), "shapes": {}}
for i, (r, v, es) in enumerate(shapes):
    grp = rows[4 * i + 1:4 * i + 4]
    kb = sorted(float(g["Counter_Value"]) for g in grp)
    name = grp[0]["Kernel_Name"].split("(")[0] if grp else "?"
    logits_kb = r * v * es / 1024
    out["shapes"][f"{r}x{v} {'f32' if es == 4 else 'bf16'}"] = {"kernel": name, "fetch_kb": kb[len(kb) // 2] if kb else None,
        "logits_kb": round(logits_kb, 1), "ratio": round(kb[len(kb) // 2] / logits_kb, 4) if kb else None}
print(json.dumps(out))
json.dump(out, open("gpurun_out/k7_pmc_fetch.json", "w"), indent=1)
PY
