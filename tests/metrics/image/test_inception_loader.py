"""Inception-v3 checkpoint loading is strict: a partial or renamed state
dict raises instead of silently leaving random weights (reference fid.py:28-50 loads
torchvision's pretrained weights; here a local checkpoint is the only source)."""

import pytest
import torch

from torcheval_amd.models.inception import inception_v3


@pytest.fixture(scope="module")
def state():
    torch.manual_seed(0)
    return inception_v3().state_dict()


def test_round_trip_and_aux_logits_dropped(tmp_path, state):
    sd = dict(state)
    sd["AuxLogits.fc.weight"] = torch.zeros(3)  # torchvision checkpoints carry the aux head
    path = tmp_path / "inc.pt"
    torch.save(sd, path)
    m = inception_v3(weights_path=str(path))
    for k, v in state.items():
        assert torch.equal(m.state_dict()[k], v), k


def test_missing_key_raises(tmp_path, state):
    sd = {k: v for k, v in state.items() if not k.startswith("Mixed_7c.")}
    path = tmp_path / "partial.pt"
    torch.save(sd, path)
    with pytest.raises(RuntimeError, match="missing keys"):
        inception_v3(weights_path=str(path))


def test_renamed_key_raises(tmp_path, state):
    sd = {("model." + k if k.startswith("fc.") else k): v for k, v in state.items()}
    path = tmp_path / "renamed.pt"
    torch.save(sd, path)
    with pytest.raises(RuntimeError, match="unexpected keys"):
        inception_v3(weights_path=str(path))
