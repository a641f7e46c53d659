"""FLOP counter and module summary (parity: tests/tools/test_flops.py, test_module_summary.py).
Pinned numbers are the reference's; the torchvision architectures are rebuilt locally."""

import copy

import pytest
import torch

from tests.tools._models import alexnet, resnet18
from torcheval_amd.tools import (
    FlopTensorDispatchMode,
    get_module_summary,
    get_summary_table,
    prune_module_summary,
)
from torcheval_amd.tools.module_summary import _get_human_readable_count


def _get(ftdm, scope, op):
    return ftdm.flop_counts[scope].get(f"{op}.default", 0) + ftdm.flop_counts[scope].get(op, 0)


def test_torch_operations() -> None:
    class M(torch.nn.Module):
        def forward(self, x):
            return x.bmm(torch.randn(10, 5, 7)).matmul(torch.randn(7, 3))

    mod = M()
    with FlopTensorDispatchMode(mod) as ftdm:
        res = mod(torch.randn(10, 4, 5))
        assert res.shape == (10, 4, 3)
        assert _get(ftdm, "", "bmm") == 1400
        assert _get(ftdm, "", "mm") == 840
        ftdm.reset()
        res = mod(torch.randn(10, 4, 5, requires_grad=True))
        res.mean().backward()
        assert _get(ftdm, "", "bmm") == 2800
        assert _get(ftdm, "", "mm") == 1680


def test_linear_layers_scoped() -> None:
    lnn = torch.nn.Sequential(
        torch.nn.Sequential(torch.nn.Linear(10, 70), torch.nn.Linear(70, 5)), torch.nn.Linear(5, 1)
    )
    with FlopTensorDispatchMode(lnn) as ftdm:
        assert len(ftdm._all_hooks) == 8
        res = lnn(torch.randn(1, 10))
        fwd = {"": 1055, "0": 1050, "0.0": 700, "0.1": 350, "1": 5}
        for k, v in fwd.items():
            assert _get(ftdm, k, "addmm") == v, k
        ftdm.reset()
        res.backward()
        bwd = {"": 1410, "0": 1400, "0.0": 700, "0.1": 700, "1": 10}
        for k, v in bwd.items():
            assert _get(ftdm, k, "mm") == v, k
    # hooks are removed on exit
    assert all(len(m._forward_hooks) == 0 for m in lnn.modules())


def test_resnet18_counts() -> None:
    mod = resnet18()
    with FlopTensorDispatchMode(mod) as ftdm:
        assert len(ftdm._all_hooks) == 2 * len(list(mod.modules())) - 2
        res = mod(torch.randn(1, 3, 224, 224))
        assert _get(ftdm, "", "convolution") == 1813561344
        assert _get(ftdm, "", "addmm") == 512000
        assert _get(ftdm, "conv1", "convolution") == 118013952
        assert _get(ftdm, "fc", "addmm") == 512000
        ftdm.reset()
        res.mean().backward()
        assert _get(ftdm, "", "convolution_backward") == 3509108736
        assert _get(ftdm, "", "mm") == 1024000
        assert _get(ftdm, "layer1", "convolution_backward") == 924844032
        assert _get(ftdm, "fc", "mm") == 1024000


def test_transposed_conv() -> None:
    m = torch.nn.ConvTranspose2d(4, 6, 3, stride=2)
    x = torch.randn(2, 4, 5, 5, requires_grad=True)
    with FlopTensorDispatchMode(m) as ftdm:
        out = m(x)
        fwd = copy.deepcopy(ftdm.flop_counts)
        ftdm.reset()
        out.sum().backward()
    macs = 2 * (4 * 6 * 9) * 25  # batch * |w| * input positions
    assert fwd[""]["convolution.default"] == macs
    assert ftdm.flop_counts[""]["convolution_backward.default"] == 2 * macs


def test_summary_layer() -> None:
    model = torch.nn.Conv2d(3, 8, 3)
    ms1 = get_module_summary(model)
    ms2 = get_module_summary(model, module_args=(torch.randn(1, 3, 8, 8),))
    assert (ms1.module_name, ms1.module_type, ms1.num_parameters) == ("", "Conv2d", 224)
    assert ms1.num_trainable_parameters == 224 and ms1.size_bytes == 224 * 4
    assert ms1.submodule_summaries == {} and not ms1.has_uninitialized_param
    assert ms2.flops_forward == 7776 and ms2.flops_backward == 7776
    assert ms1.in_size == "?" and ms1.out_size == "?"
    assert ms2.in_size == [1, 3, 8, 8] and ms2.out_size == [1, 8, 6, 6]
    expect = (
        "Name | Type   | # Parameters | # Trainable Parameters | Size (bytes) | Contains Uninitialized Parameters?\n"
        "---------------------------------------------------------------------------------------------------------\n"
        "     | Conv2d | 224          | 224                    | 896          | No"
    )
    for a, b in zip(expect.split("\n"), str(ms1).strip().split("\n")):
        assert a.strip() == b.strip()


def test_activation_sizes() -> None:
    class M(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.hidden = torch.nn.Linear(10, 5)
            self.relu = torch.nn.ReLU()
            self.out = torch.nn.Linear(5, 3)
            self.softmax = torch.nn.Softmax(dim=3)

        def forward(self, x):
            return self.softmax(self.out(self.relu(self.hidden(x))))

    ms = get_module_summary(M(), (torch.randn(1, 3, 10, 10),))
    assert ms.in_size == [1, 3, 10, 10] and ms.out_size == [1, 3, 10, 3]
    sub = ms.submodule_summaries
    assert sub["hidden"].out_size == [1, 3, 10, 5] and sub["hidden"].module_type == "Linear"
    assert sub["relu"].in_size == [1, 3, 10, 5]
    assert sub["softmax"].out_size == [1, 3, 10, 3]


def test_prune_and_lazy() -> None:
    summary = get_module_summary(torch.nn.Conv2d(3, 8, 3))
    with pytest.raises(ValueError, match="Got -2."):
        prune_module_summary(summary, max_depth=-2)
    with pytest.raises(ValueError, match="Got 0."):
        prune_module_summary(summary, max_depth=0)
    ms = get_module_summary(torch.nn.LazyLinear(10), module_args=(torch.randn(1, 10),))
    with pytest.warns(Warning):
        ms.num_parameters
    assert ms.has_uninitialized_param and ms.flops_forward == "?" and ms.flops_backward == "?"


def test_resnet_depth_and_flops() -> None:
    model = resnet18()
    ms1 = get_module_summary(model)
    assert len(ms1.submodule_summaries) == 10
    assert len(ms1.submodule_summaries["layer2"].submodule_summaries) == 2
    assert len(ms1.submodule_summaries["layer2"].submodule_summaries["layer2.0"].submodule_summaries) == 6
    ms4 = get_module_summary(model, module_args=(torch.randn(1, 3, 224, 224),))
    prune_module_summary(ms4, max_depth=2)
    assert ms4.flops_forward == 1814073344
    assert ms4.flops_backward == 3510132736
    assert ms4.submodule_summaries["layer2"].flops_forward == 411041792
    assert ms4.submodule_summaries["layer2"].flops_backward == 822083584
    assert ms4.num_parameters == 11689512


def test_alexnet_tables_and_times() -> None:
    model = alexnet()
    ms = get_module_summary(model)
    prune_module_summary(ms, max_depth=2)
    expect = (
        "Name       | Type              | # Parameters | # Trainable Parameters | Size (bytes) | Contains Uninitialized Parameters?\n"
        "--------------------------------------------------------------------------------------------------------------------------\n"
        "           | AlexNet           | 61.1 M       | 61.1 M                 | 244 M        | No\n"
        "features   | Sequential        | 2.5 M        | 2.5 M                  | 9.9 M        | No\n"
        "avgpool    | AdaptiveAvgPool2d | 0            | 0                      | 0            | No\n"
        "classifier | Sequential        | 58.6 M       | 58.6 M                 | 234 M        | No"
    )
    for a, b in zip(expect.split("\n"), str(ms).strip().split("\n")):
        assert a.strip() == b.strip()
    inp = torch.randn(1, 3, 224, 224)
    ms = get_module_summary(model, module_args=(inp,))
    assert ms.flops_forward == 714188480 and ms.flops_backward == 1358100160
    feats = ms.submodule_summaries["features"]
    assert feats.flops_forward == 655566528 and feats.flops_backward == 1240856256
    assert feats.out_size == [1, 256, 6, 6]
    cls = ms.submodule_summaries["classifier"]
    assert cls.flops_forward == 58621952 and cls.flops_backward == 117243904
    stack = [ms]
    while stack:
        s = stack.pop()
        assert s.forward_elapsed_time_ms != "?" and float(s.forward_elapsed_time_ms) > 0
        stack.extend(s.submodule_summaries.values())
    # real milliseconds: the whole forward of AlexNet on CPU takes well over 0.01 ms
    assert ms.forward_elapsed_time_ms > 0.01
    assert "Forward FLOPs" in get_summary_table(ms) and "Remark for FLOPs" in get_summary_table(ms)


def test_multiple_inputs() -> None:
    class SimpleConv(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.features = torch.nn.Sequential(
                torch.nn.Conv2d(1, 1, kernel_size=3, stride=1, padding=1), torch.nn.ReLU(inplace=True)
            )

        def forward(self, x, y):
            return torch.cat((self.features(x), self.features(y)), 1)

    x, y = torch.randn(1, 1, 64, 64), torch.randn(1, 1, 64, 64)
    ms = get_module_summary(SimpleConv(), module_args=(x, y))
    assert ms.num_parameters == 10
    assert ms.in_size == [[1, 1, 64, 64], [1, 1, 64, 64]] and ms.out_size == [1, 2, 64, 64]
    relu = ms.submodule_summaries["features"].submodule_summaries["features.1"]
    assert relu.flops_forward == 0 and relu.flops_backward == 0


def test_human_readable() -> None:
    with pytest.raises(ValueError, match="received -1"):
        _get_human_readable_count(-1)
    with pytest.raises(TypeError, match="received <class 'float'>"):
        _get_human_readable_count(0.1)
    cases = {1: "1  ", 123: "123  ", 1234: "1.2 K", 1254: "1.3 K", 1960: "2.0 K", 10**4: "10.0 K",
             10**6: "1.0 M", 10**9: "1.0 B", 10**12: "1.0 T", 10**15: "1,000 T"}
    for n, s in cases.items():
        assert _get_human_readable_count(n) == s
