"""bench.py contract: the timed region runs nothing that the warmup did not already run.

Round 1's driver run (--steps 20 --warmup 5) timed the first-ever ``compute()`` (a lazy
kernel-object load) inside a 20-step region and reported 424 updates/s instead of ~110k.
This test pins the structure that prevents it: warmup and the timed region both call the
same ``run()`` (updates + compute / sync_and_compute), and the timed region calls nothing else
besides synchronisation.
"""

import ast
import os

BENCH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench.py")


def _main_body():
    tree = ast.parse(open(BENCH).read())
    main = next(n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name == "main")
    return main


def _calls(nodes):
    out = []
    for n in nodes:
        for c in ast.walk(n):
            if isinstance(c, ast.Call):
                out.append(ast.unparse(c.func))
    return out


def test_timed_region_only_runs_the_warmed_sequence():
    main = _main_body()
    body = main.body
    # the timed region: from `t0 = time.perf_counter()` to `elapsed = ...`
    start = next(i for i, s in enumerate(body) if isinstance(s, ast.Assign)
                 and ast.unparse(s.targets[0]) == "t0")
    stop = next(i for i, s in enumerate(body) if isinstance(s, ast.Assign)
                and ast.unparse(s.targets[0]) == "elapsed")
    timed = _calls(body[start + 1:stop])
    assert "run" in timed
    allowed = {"run", "device_sync"}  # the closing rendezvous is run()'s sync_and_compute
    assert set(timed) <= allowed, set(timed) - allowed
    # the warmup (before t0) calls the same run() and synchronises
    warm = _calls(body[:start])
    assert "run" in warm and "metric.reset" in warm
    # barrier + device synchronize right before t0
    assert _calls(body[start - 2:start]) == ["barrier", "device_sync"]


def test_run_includes_compute():
    main = _main_body()
    run = next(n for n in ast.walk(main) if isinstance(n, ast.FunctionDef) and n.name == "run")
    calls = _calls(run.body)
    assert "metric.update" in calls
    assert "metric.compute" in calls and "sync_and_compute" in calls
