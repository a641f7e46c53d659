"""Runtime flags: read once from the environment, settable at runtime.

=============================  ========================================================
``TORCHEVAL_AMD_DISABLE_HIP``  1: run the ATen path even for ROCm tensors (debug / A-B)
``TORCHEVAL_AMD_VALIDATE``     1: raise input-validation errors at the ``update()`` that
                               caused them (one host sync per update), like the reference;
                               0 (default): kernels record violations in a device flag
                               that ``compute()`` raises (no per-update sync)
``TORCHEVAL_AMD_DETERMINISTIC``  1: reductions whose float accumulation order depends on
                               block scheduling (K6 entropy sums, K7 perplexity sums) use
                               an ordered two-pass fold - bit-identical run to run
``TORCHEVAL_AMD_TRACE``        1: ``torch.profiler.record_function`` ranges around every
                               metric ``update`` / ``compute`` / ``merge_state`` and the
                               toolkit syncs (visible in torch.profiler and rocprofv3 -r)
=============================  ========================================================

Use ``torcheval_amd.config.flags(validate=True)`` as a context manager for a scoped change.
``deterministic`` also keeps multi-rank syncs on the rank-ordered gather + ``seg_reduce`` path
(``parallel/rccl_direct.py``).

Engine policies (read once per process; not flags):

=============================================  ==============================================
``TORCHEVAL_AMD_DIRECT_RCCL``                  ``auto`` (default): the engine's own RCCL
                                               communicators for 1-rank groups only; ``1``:
                                               every group; ``0``: always torch.distributed
``TORCHEVAL_AMD_RCCL_ASYNC_ERROR_HANDLING``    1 (default): a failed direct communicator ends
                                               the process (c10d's default); 0: the next sync
                                               votes group-wide and rebuilds - the vote is a
                                               blocking torch.distributed MIN all-reduce + a
                                               host read before EVERY direct sync at ws > 1
                                               (async side-stream syncs included, which then
                                               synchronise the host once per call)
``TORCHEVAL_AMD_ASYNC_DIRECT_RCCL``            1: async syncs ride the direct path on a side
                                               stream (default: torch.distributed async)
``TORCHEVAL_AMD_RCCL_WATCHDOG``                0: no completion watchdog (A/B only)
``TORCHEVAL_AMD_HOST_POLL_US``                 bound of the pinned-memory host spin of device
                                               flag reads (``ops/hostread.py``)
=============================================  ==============================================

Kernel A/B knobs (benchmarks only; defaults are the measured winners, ``profiles/README.md``):
``TORCHEVAL_AMD_K1_MICRO`` / ``_K1_WPB`` (K1 micro kernel, waves per workgroup),
``_K3_ONESWEEP`` (0: the upsweep / downsweep sort), ``_K3_ROUNDS`` (8 / 16 keys per thread),
``_K3_HIST_ROUNDS`` (onesweep histogram rounds per block), ``_K3_FOLD`` (1: tile sums folded into
the last onesweep pass, 7 launches, measured slower) / ``_K3_FOLD_PROBE``, ``_K5_V2 / ``_K5_CG`` / ``_K5_MAXR`` /
``_K5_BLOCKS`` / ``_K5_PIPE`` / ``_K5_AB_SKIP_FOLD`` (K5 geometry; read per call only with
``_AB_DYNAMIC``), ``_K5B_MODE`` / ``_K5B_GRID`` / ``_K5B_PEND_VPT`` (K5b launch shape),
``_K8_MODE`` / ``_K8_SPLIT`` / ``_K8_EXACT`` / ``_FID_STAGE_ROWS`` (FID covariance),
``_PPL_U2`` / ``_PPL_MAXGRID`` (K7), ``_SYMEIG_COOP`` (K9b cooperative launch), ``_SYMEIG_WAVE``
(1: the rows-per-wave K9b reduction, measured slower),
``_MAX_BLOCKS`` (grid cap), ``_ARCH`` (build target, default gfx950).
"""

import contextlib
import os
from typing import Iterator


def _env(name: str) -> bool:
    return os.environ.get(name, "0") not in ("", "0", "false", "False")


class _Config:
    __slots__ = ("validate", "deterministic", "trace")

    def __init__(self) -> None:
        self.validate = _env("TORCHEVAL_AMD_VALIDATE")
        self.deterministic = _env("TORCHEVAL_AMD_DETERMINISTIC")
        self.trace = _env("TORCHEVAL_AMD_TRACE")

    @property
    def disable_hip(self) -> bool:
        from torcheval_amd import ops

        return ops.DISABLE_HIP

    @disable_hip.setter
    def disable_hip(self, value: bool) -> None:
        from torcheval_amd import ops

        ops.DISABLE_HIP = bool(value)

    def __repr__(self) -> str:
        return (
            f"config(disable_hip={self.disable_hip}, validate={self.validate}, "
            f"deterministic={self.deterministic}, trace={self.trace})"
        )


config = _Config()


@contextlib.contextmanager
def flags(**kwargs: bool) -> Iterator[_Config]:
    """Temporarily set flags: ``with flags(validate=True, deterministic=True): ...``."""
    old = {k: getattr(config, k) for k in kwargs}
    try:
        for k, v in kwargs.items():
            if not hasattr(type(config), k) and k not in _Config.__slots__:
                raise AttributeError(f"unknown flag {k!r}")
            setattr(config, k, v)
        yield config
    finally:
        for k, v in old.items():
            setattr(config, k, v)


def trace_range(name: str):
    """``record_function(name)`` when tracing is on, else a no-op context."""
    if config.trace:
        import torch

        return torch.profiler.record_function(name)
    return contextlib.nullcontext()


__all__ = ["config", "flags", "trace_range"]
