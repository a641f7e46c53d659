"""a onesweep look-back timeout is surfaced, never a silent wrong AUC.  With
the spin limit forced to 1 poll (TORCHEVAL_AMD_K3_SPIN_LIMIT, read once per process: a child
process), tiles give up on predecessors that have not published yet: the scan of that sort returns
NaN (never a wrong finite value), the next sort warns and every later sort of the process takes
the legacy radix passes, whose results are exact again."""

import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

_CHILD = r"""
import warnings
import torch
from torcheval_amd.metrics.functional import binary_auroc
from torcheval_amd.ops import native
g = torch.Generator().manual_seed(0)
x, t = torch.rand(1_000_000, generator=g), torch.randint(0, 2, (1_000_000,), generator=g)
ref = float(binary_auroc(x, t))
xd, td = x.cuda(), t.cuda()
first = float(binary_auroc(xd, td))
flag = native().sort_desc_timeouts(xd, False)
with warnings.catch_warnings(record=True) as w:
    warnings.simplefilter("always")
    later = [float(binary_auroc(xd, td)) for _ in range(3)]
import json
print(json.dumps([ref, first, flag, later, [str(x.message) for x in w]]))
"""


def test_forced_timeout_is_nan_then_legacy():
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    env = dict(os.environ, TORCHEVAL_AMD_K3_SPIN_LIMIT="1")
    r = subprocess.run([sys.executable, "-c", _CHILD], env=env, cwd=root, capture_output=True, text=True,
                       timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    import json

    ref, first, flag, later, warns = json.loads(r.stdout.strip().splitlines()[-1])
    assert first != first or abs(first - ref) < 1e-6  # NaN when it timed out, never a wrong number
    if flag or first != first:
        assert any("legacy radix passes" in m for m in warns), warns
    # once a timeout was seen the process sorts through the legacy passes: exact again
    for v in later[1:]:
        assert abs(v - ref) < 1e-6, (v, ref)
