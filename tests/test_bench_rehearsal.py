"""The driver's exact N=8 launch of bench.py (torch.distributed.run, 8 processes, 127.0.0.1)
rehearsed on CPU tensors over gloo: every rank runs the multi-rank timed region (updates +
sync_and_compute through the state-buffer engine) and rank 0 prints the one JSON line."""

import json
import os
import socket
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_bench_8_rank_launch_on_cpu():
    env = dict(os.environ, BENCH_DEVICE="cpu", BENCH_EXTRAS="sync", OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py",
           "--gpus", "8", "--steps", "3", "--warmup", "1"]
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 8 and out["steps"] == 3 and out["warmup"] == 1
    assert out["config"]["parallelism"] == "dp8" and out["config"]["global_batch"] == 8 * 8192
    assert out["value"] > 0 and out["higher_is_better"] is True and out["scaling"] == "weak"
    assert "CPU rehearsal" in out["data"]
    # N > 1 diagnostics: the headline's own closing sync, the path it took,
    # and the direct-RCCL arm - timed, or its voted fallback (gloo: no direct communicator)
    sync = out["sync_ms"]
    assert isinstance(sync, dict), sync
    for key in ("accuracy_sync_and_compute", "confusion_matrix_1000_sync_and_compute",
                "direct_accuracy_sync_and_compute", "direct_confusion_matrix_1000_sync_and_compute"):
        assert isinstance(sync[key], float) and sync[key] > 0, (key, sync[key])
    assert sync["sync_path"] == "c10d"
    assert sync["direct_sync_path"] in ("direct-rccl", "c10d")
