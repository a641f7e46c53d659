"""The examples run and reproduce the reference's golden output."""

import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_simple_example_golden_line() -> None:
    sys.path.insert(0, os.path.join(REPO, "examples"))
    import simple_example

    assert simple_example.main("cpu") == "Epoch 4/4, Batch 16/16 --- loss: 0.6268, acc: 0.6094"


def test_distributed_example_gloo() -> None:
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="1")
    out = subprocess.run(
        [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
         "--master-addr", "127.0.0.1", "--master-port", "29561",
         os.path.join(REPO, "examples", "distributed_example.py"), "--device", "cpu"],
        env=env, capture_output=True, text=True, timeout=300,
    )
    assert out.returncode == 0, out.stderr[-2000:]
    assert "Epoch 4/4, Batch 16/16" in out.stdout
    assert "synced throughput" in out.stdout


def test_tour_runs() -> None:
    from examples import tour  # importable by the gloo worker processes (repo root on sys.path)

    tour.main("cpu")
