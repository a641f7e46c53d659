"""Persistent multi-process gloo worker pool for distributed CPU tests.

The reference spawns a fresh elastic launch (4 processes, c10d rendezvous) for every class
test (metric_class_tester.py:292-312).  Process start-up (importing torch) dominates that,
so here one pool of ``world_size`` ranks is started lazily per world size and reused by every
test of the session.  A job is a picklable callable ``fn(rank, world_size, *args)`` run on
every rank at once; results come back in rank order, and any rank's exception is re-raised
in the parent with its traceback.  A job that does not finish in ``timeout`` seconds (e.g. a
rank died mid-collective) kills the pool; the next job starts a new one.
"""

import atexit
import os
import queue
import socket
import traceback
from typing import Any, Callable, Dict, List, Tuple

import torch.multiprocessing as mp


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank: int, world_size: int, port: int, jobs, results) -> None:
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["RANK"] = str(rank)
    os.environ["LOCAL_RANK"] = str(rank)
    os.environ["WORLD_SIZE"] = str(world_size)
    os.environ.setdefault("OMP_NUM_THREADS", "1")
    import torch
    import torch.distributed as dist

    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world_size)
    while True:
        job = jobs.get()
        if job is None:
            break
        job_id, fn, args = job
        try:
            out = fn(rank, world_size, *args)
            results.put((job_id, rank, True, out))
        except BaseException:  # noqa: B902 - report everything to the parent
            results.put((job_id, rank, False, traceback.format_exc()))
    dist.destroy_process_group()


class DistWorkerPool:
    def __init__(self, world_size: int) -> None:
        self.world_size = world_size
        ctx = mp.get_context("spawn")
        self._results = ctx.Queue()
        self._jobs = [ctx.Queue() for _ in range(world_size)]
        port = _free_port()
        self._procs = [
            ctx.Process(target=_worker, args=(r, world_size, port, self._jobs[r], self._results), daemon=True)
            for r in range(world_size)
        ]
        for p in self._procs:
            p.start()
        self._next_id = 0

    def alive(self) -> bool:
        return all(p.is_alive() for p in self._procs)

    def run(self, fn: Callable[..., Any], *args: Any, timeout: float = 180.0) -> List[Any]:
        job_id = self._next_id
        self._next_id += 1
        for q in self._jobs:
            q.put((job_id, fn, args))
        out: Dict[int, Any] = {}
        errors: List[Tuple[int, str]] = []
        while len(out) + len(errors) < self.world_size:
            try:
                # once a rank has failed, the others may be stuck in a collective
                jid, rank, ok, payload = self._results.get(timeout=20.0 if errors else timeout)
            except queue.Empty:
                self.close(force=True)
                if errors:
                    rank, tb = sorted(errors)[0]
                    raise AssertionError(f"rank {rank} failed (pool reset):\n{tb}")
                raise TimeoutError(f"distributed test job timed out after {timeout}s")
            if jid != job_id:
                continue
            if ok:
                out[rank] = payload
            else:
                errors.append((rank, payload))
        if errors:
            rank, tb = sorted(errors)[0]
            raise AssertionError(f"rank {rank} failed:\n{tb}")
        return [out[r] for r in range(self.world_size)]

    def close(self, force: bool = False) -> None:
        if not force:
            for q in self._jobs:
                try:
                    q.put(None)
                except Exception:
                    pass
            for p in self._procs:
                p.join(timeout=10)
        for p in self._procs:
            if p.is_alive():
                p.kill()
                p.join(timeout=5)


_POOLS: Dict[int, DistWorkerPool] = {}


def get_pool(world_size: int) -> DistWorkerPool:
    pool = _POOLS.get(world_size)
    if pool is None or not pool.alive():
        if pool is not None:
            pool.close(force=True)
        pool = DistWorkerPool(world_size)
        _POOLS[world_size] = pool
    return pool


def run_distributed(fn: Callable[..., Any], world_size: int, *args: Any, timeout: float = 180.0) -> List[Any]:
    """Run ``fn(rank, world_size, *args)`` on every rank of a gloo world; rank-ordered results."""
    pool = get_pool(world_size)
    try:
        return pool.run(fn, *args, timeout=timeout)
    except TimeoutError:
        _POOLS.pop(world_size, None)
        raise


@atexit.register
def _shutdown() -> None:
    for pool in list(_POOLS.values()):
        pool.close()
    _POOLS.clear()
