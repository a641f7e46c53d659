"""binary_auroc at N=1M (BASELINE config 3): wall time per call for the K3 variants - the
onesweep sort (TORCHEVAL_AMD_K3_ONESWEEP) and tile_sums folded into tile_area
(TORCHEVAL_AMD_K3_LB), each against its legacy form.  The variables are read once per process,
so each mode runs in its own child process; one JSON line per mode."""
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
res["auroc_abs_err_vs_cpu"] = abs(float(binary_auroc(x, t).cpu()) - float(binary_auroc(x.cpu().double(), t.cpu())))
res["auprc_abs_err_vs_cpu"] = abs(float(binary_auprc(x, t).cpu()) - float(binary_auprc(x.cpu().double(), t.cpu())))
print(json.dumps(res))
'''

repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for mode, lb, dyn in (("1", "0", "0"), ("1", "1", "0"), ("0", "0", "0")):
    env = dict(os.environ, TORCHEVAL_AMD_K3_ONESWEEP=mode, TORCHEVAL_AMD_K3_LB=lb, TORCHEVAL_AMD_K3_DYNID=dyn, REPO=repo)
    out = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
    if out.returncode != 0:
        print(out.stdout[-2000:], out.stderr[-4000:])
        sys.exit(out.returncode)
    line = json.loads(out.stdout.strip().splitlines()[-1])
    line["onesweep"] = mode == "1"
    line["tile_sums_folded"] = lb == "1"
    line["tile_ids"] = "counter" if dyn == "1" else "blockIdx"
    line["n"] = int(os.environ.get("AUROC_N", "1000000"))
    print(json.dumps(line), flush=True)
