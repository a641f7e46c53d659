"""Inputs past 2^31 elements (and other large shapes) on one MI355X: the HIP kernels against the
ATen path of the same functions (``config.disable_hip``) on the same device.  These pin the
64-bit index arithmetic of K1 / K3 / K4 / K5 / K7, which the small parity cases never reach."""

import contextlib

import pytest
import torch

from torcheval_amd.config import config
from torcheval_amd.metrics import functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


@contextlib.contextmanager
def _aten():
    old = config.disable_hip
    config.disable_hip = True
    try:
        yield
    finally:
        config.disable_hip = old


def _free():
    torch.cuda.synchronize()
    torch.cuda.empty_cache()


def test_k1_accuracy_over_2g_elements():
    g = torch.Generator(device=DEV).manual_seed(0)
    x = torch.randn(25_000, 100_000, device=DEV, generator=g)  # 2.5e9 logits, 10 GB
    y = torch.randint(0, 100_000, (25_000,), device=DEV, generator=g)
    y[::3] = x[::3].argmax(dim=1)  # a third correct
    got = F.multiclass_accuracy(x, y)
    with _aten():
        exp = F.multiclass_accuracy(x, y)
    torch.testing.assert_close(got.cpu(), exp.cpu())
    del x
    _free()


def test_k3_binary_auroc_33m_with_ties():
    g = torch.Generator(device=DEV).manual_seed(1)
    n = (1 << 25) + 7
    x = torch.randint(0, 5000, (n,), device=DEV, generator=g).float() / 5000
    t = torch.randint(0, 2, (n,), device=DEV, generator=g)
    got_roc, got_pr = F.binary_auroc(x, t), F.binary_auprc(x, t)
    with _aten():
        exp_roc, exp_pr = F.binary_auroc(x, t), F.binary_auprc(x, t)
    torch.testing.assert_close(got_roc.cpu(), exp_roc.cpu(), rtol=1e-6, atol=1e-9)
    torch.testing.assert_close(got_pr.cpu(), exp_pr.cpu(), rtol=1e-5, atol=1e-7)
    _free()


def test_k4_binned_300m_elements():
    g = torch.Generator(device=DEV).manual_seed(2)
    n, c = 3_000_000, 100
    x = torch.rand(n, c, device=DEV, generator=g)
    y = torch.randint(0, c, (n,), device=DEV, generator=g)
    got = F.multiclass_binned_auprc(x, y, num_classes=c, threshold=100, average=None)
    with _aten():
        exp = F.multiclass_binned_auprc(x, y, num_classes=c, threshold=100, average=None)
    for a, b in zip(got, exp):
        torch.testing.assert_close(a.cpu(), b.cpu(), rtol=1e-5, atol=1e-6)
    del x
    _free()


def test_k5_mse_r2_over_2g_elements():
    g = torch.Generator(device=DEV).manual_seed(3)
    x = torch.rand(50_000, 44_000, device=DEV, generator=g)  # 2.2e9 elements each
    t = x + 0.1 * torch.randn(50_000, 44_000, device=DEV, generator=g)
    got_mse = F.mean_squared_error(x, t)
    got_r2 = F.r2_score(x, t)
    # ATen reference in float64 column chunks (an fp32 torch.mean over 2.2e9 terms would be
    # the least accurate party here)
    sse = torch.zeros(44_000, dtype=torch.float64, device=DEV)
    st = torch.zeros_like(sse)
    stt = torch.zeros_like(sse)
    for r0 in range(0, 50_000, 5_000):
        xs, ts = x[r0:r0 + 5_000].double(), t[r0:r0 + 5_000].double()
        sse += ((ts - xs) ** 2).sum(0)
        st += ts.sum(0)
        stt += (ts * ts).sum(0)
    exp_mse = (sse / 50_000).mean()
    exp_r2 = (1 - sse / (stt - st * st / 50_000)).mean()
    torch.testing.assert_close(got_mse.double().cpu(), exp_mse.cpu(), rtol=1e-4, atol=0)
    torch.testing.assert_close(got_r2.double().cpu(), exp_r2.cpu(), rtol=1e-4, atol=1e-5)
    del x, t
    _free()


def test_k7_perplexity_over_2g_logits():
    g = torch.Generator(device=DEV).manual_seed(4)
    logits = torch.randn(2, 8192, 150_000, device=DEV, generator=g)  # 2.46e9 logits, 9.8 GB
    tok = torch.randint(0, 150_000, (2, 8192), device=DEV, generator=g)
    got = F.perplexity(logits, tok)
    # reference: log-softmax row by row in float64 chunks
    nll = torch.zeros((), dtype=torch.float64, device=DEV)
    flat, ft = logits.view(-1, 150_000), tok.view(-1)
    for r0 in range(0, flat.shape[0], 1024):
        lp = torch.log_softmax(flat[r0:r0 + 1024].double(), dim=1)
        nll -= lp.gather(1, ft[r0:r0 + 1024, None]).sum()
    exp = torch.exp(nll / flat.shape[0])
    torch.testing.assert_close(got.double().cpu(), exp.cpu(), rtol=1e-5, atol=0)
    del logits, flat
    _free()
