"""Run the `run:` steps of a GitHub workflow job locally and record the outcome.

    python ci/run_workflow.py .github/workflows/unit_test.yaml cpu --out profiles/ci_cpu_job_r2.json
    python ci/run_workflow.py .github/workflows/unit_test.yaml mi355x --skip build   # on the GPU box

The workflows themselves need GitHub runners (an ubuntu container and a self-hosted MI355X);
this executes the same commands in this repository's environment so the steps are known to
pass as written.  ``--skip`` drops steps whose name or command contains the given text (e.g.
a `pip install` with no package index, or a rebuild of an extension that is already built).
"""

import argparse
import json
import subprocess
import sys
import time

import yaml


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("workflow")
    ap.add_argument("job")
    ap.add_argument("--skip", action="append", default=[])
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    with open(args.workflow) as f:
        wf = yaml.safe_load(f)
    steps = wf["jobs"][args.job]["steps"]
    record = {"workflow": args.workflow, "job": args.job, "steps": []}
    rc_all = 0
    for i, st in enumerate(steps):
        cmd = st.get("run")
        name = st.get("name", cmd or st.get("uses", f"step {i}"))
        if cmd is None:
            record["steps"].append({"name": name, "status": "not a run step (uses: %s)" % st.get("uses")})
            continue
        if any(s in name or s in cmd for s in args.skip):
            record["steps"].append({"name": name, "cmd": cmd, "status": "skipped"})
            continue
        t0 = time.perf_counter()
        p = subprocess.run(["bash", "-o", "pipefail", "-c", cmd], capture_output=True, text=True)
        dt = time.perf_counter() - t0
        tail = (p.stdout.strip() or p.stderr.strip()).splitlines()[-3:]
        record["steps"].append({"name": name, "cmd": cmd, "rc": p.returncode, "seconds": round(dt, 1), "tail": tail})
        print(f"[{p.returncode}] {name} ({dt:.1f}s): {tail[-1] if tail else ''}", flush=True)
        if p.returncode != 0:
            rc_all = p.returncode
            break
    record["passed"] = rc_all == 0
    if args.out:
        with open(args.out, "w") as f:
            json.dump(record, f, indent=1)
    return rc_all


if __name__ == "__main__":
    sys.exit(main())
