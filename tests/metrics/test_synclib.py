import torch

from torcheval_amd.metrics.synclib import metrics_traversal_order, sync_states
from torcheval_amd.utils.test_utils import run_distributed


def _sync(rank, ws):
    states = {
        "m2": {"t": torch.tensor([rank, rank + 1.0]), "n": rank, "f": float(rank) / 2},
        "m1": {
            "l": [torch.full((rank + 1, 2), float(rank)) for _ in range(rank)],  # rank 0: empty
            "d": {"a": torch.tensor(float(rank))},
        },
    }
    order = metrics_traversal_order(states)
    out = sync_states(states, {"m1": torch.device("cpu"), "m2": torch.device("cpu")}, order)
    return order, out


def test_sync_states_all_kinds():
    res = run_distributed(_sync, 3)
    for order, out in res:
        assert order == [("m1", "d"), ("m1", "l"), ("m2", "f"), ("m2", "n"), ("m2", "t")]
        assert len(out) == 3
        for r in range(3):
            torch.testing.assert_close(out[r]["m2"]["t"], torch.tensor([r, r + 1.0]))
            assert out[r]["m2"]["n"] == r and out[r]["m2"]["f"] == r / 2
            assert len(out[r]["m1"]["l"]) == r
            for t in out[r]["m1"]["l"]:
                torch.testing.assert_close(t, torch.full((r + 1, 2), float(r)))
            torch.testing.assert_close(out[r]["m1"]["d"]["a"], torch.tensor(float(r)))
