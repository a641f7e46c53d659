"""binary_auroc at N=1M (BASELINE config 3): wall time per call, onesweep sort vs the legacy
upsweep / downsweep sort (TORCHEVAL_AMD_K3_ONESWEEP=0).  The variable is read once per process,
so each mode runs in its own child process; one JSON line per mode.  TORCHEVAL_AMD_K3_FOLD=1
turns on the tile-sum fold into the last onesweep pass (no tile_sums launch); K3_AB_FOLD_PROBE=1
splits its cost (TORCHEVAL_AMD_K3_FOLD_PROBE: 1 = no atomics, 2 = no fold work).  (Round 5 also measured a
tile_sums fold into tile_area and counter-ticket tile ids - both slower and removed:
profiles/k3_onesweep_r5.json.)"""
import json
import os
import subprocess
import sys

CHILD = r'''
import json, os, sys, torch
sys.path.insert(0, os.environ["REPO"])
from torcheval_amd.metrics.functional import binary_auroc, binary_auprc
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(0)
n = int(os.environ.get("AUROC_N", "1000000"))
x = torch.rand(n, device=dev, generator=g)
t = torch.randint(0, 2, (n,), device=dev, generator=g)
for _ in range(20):
    binary_auroc(x, t)
torch.cuda.synchronize()
res = {}
for name, fn in (("binary_auroc", binary_auroc), ("binary_auprc", binary_auprc)):
    reps = []
    for _ in range(7):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(50):
            fn(x, t)
        e.record()
        torch.cuda.synchronize()
        reps.append(s.elapsed_time(e) / 50 * 1e3)
    reps.sort()
    res[name] = {"median_us": round(reps[3], 2), "min_us": round(reps[0], 2)}
xm = torch.rand(100_000, 100, device=dev, generator=g)
ym = torch.randint(0, 100, (100_000,), device=dev, generator=g)
from torcheval_amd.metrics.functional import multiclass_auroc
for _ in range(5):
    multiclass_auroc(xm, ym, num_classes=100)
reps = []
for _ in range(7):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(10):
        multiclass_auroc(xm, ym, num_classes=100)
    e.record()
    torch.cuda.synchronize()
    reps.append(s.elapsed_time(e) / 10 * 1e3)
reps.sort()
res["multiclass_auroc_100k_x100"] = {"median_us": round(reps[3], 2), "min_us": round(reps[0], 2)}
res["auroc_abs_err_vs_cpu"] = abs(float(binary_auroc(x, t).cpu()) - float(binary_auroc(x.cpu().double(), t.cpu())))
res["auprc_abs_err_vs_cpu"] = abs(float(binary_auprc(x, t).cpu()) - float(binary_auprc(x.cpu().double(), t.cpu())))
print(json.dumps(res))
'''

repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MODES = [("1", "", "1"), ("1", "", "0"), ("0", "", "1")]
if os.environ.get("K3_AB_FOLD_PROBE") == "1":  # fold cost split: no atomics / no fold work at all
    MODES = [("1", "", "1"), ("1", "", "1p1"), ("1", "", "1p2"), ("1", "", "0")]
HIST = [h for h in os.environ.get("K3_AB_HIST_ROUNDS", "").split(",") if h]
if HIST:  # histogram blocks of 4096 x h keys (TORCHEVAL_AMD_K3_HIST_ROUNDS), default sort otherwise
    MODES = [("1", "", "0h" + h) for h in HIST]
if os.environ.get("K3_AB_ROUNDS") == "1":
    MODES += [("1", "16", "1"), ("0", "16", "1")]
if os.environ.get("K3_AB_BUCKET") == "1":  # splitter-bucket mode (default) vs the four onesweep passes
    MODES = [("1", "", "0b1"), ("1", "", "0b0"), ("1", "", "0b1"), ("1", "", "0b0")]
for mode, rounds, fold in MODES:
    env = dict(os.environ, TORCHEVAL_AMD_K3_ONESWEEP=mode, TORCHEVAL_AMD_K3_ROUNDS=rounds,
               TORCHEVAL_AMD_K3_FOLD=fold[0], REPO=repo)
    if fold[1:2] == "p":
        env["TORCHEVAL_AMD_K3_FOLD_PROBE"] = fold[2:]
    if fold[1:2] == "h":
        env["TORCHEVAL_AMD_K3_HIST_ROUNDS"] = fold[2:]
    if fold[1:2] == "b":
        env["TORCHEVAL_AMD_K3_BUCKET"] = fold[2:]
    out = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
    if out.returncode != 0:
        print(out.stdout[-2000:], out.stderr[-4000:])
        sys.exit(out.returncode)
    line = json.loads(out.stdout.strip().splitlines()[-1])
    line["onesweep"] = mode == "1"
    line["rounds"] = rounds or "default"
    line["tile_sums_fold"] = fold[0] == "1" and mode == "1"
    line["fold_probe"] = fold[2:] if fold[1:2] == "p" else None
    line["hist_rounds"] = fold[2:] if fold[1:2] == "h" else "1"
    line["bucket"] = fold[2:] != "0" if fold[1:2] == "b" else None
    line["n"] = int(os.environ.get("AUROC_N", "1000000"))
    print(json.dumps(line), flush=True)
