"""Every class case of ``cases.py`` synced through the multi-rank engine on a 1-rank ``nccl``
group on cuda:0 (``collectives_at_world_size_1``): the direct-RCCL plan of every state layout
(sum / max / min groups, bool and wide dtypes, device error flags) or the torch.distributed
path where a layout has no plan, and ``sync_and_compute`` must still reproduce the reference's
own golden result.  (Reference call stack: toolkit.py:206-260.)"""

import os
import socket
import sys

import pytest
import torch
import torch.distributed as dist

HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)

import cases  # noqa: E402
from test_parity import GOLDEN, _check, _to  # noqa: E402

import torcheval_amd.metrics as M  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture(scope="module")
def pg():
    if dist.is_initialized():
        pytest.skip("a default process group already exists in this process")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                            device_id=DEV)
    yield dist.group.WORLD
    from torcheval_amd.parallel import rccl_direct

    torch.cuda.synchronize()
    rccl_direct.destroy_all()
    dist.destroy_process_group()


@pytest.mark.parametrize("cid", sorted(cases.CLASS))
def test_class_sync_and_compute_rccl(pg, cid):
    from torcheval_amd.metrics.toolkit import sync_and_compute
    from torcheval_amd.parallel.collectives import collectives_at_world_size_1

    cls_name, ctor, upd = cases.CLASS[cid]
    updates = _to(upd(cases.cid_seed(cid)), DEV)

    def run():
        m = getattr(M, cls_name)(**ctor(), device=DEV)
        for args, kwargs in updates:
            m.update(*args, **kwargs)
        with collectives_at_world_size_1():
            return sync_and_compute(m)

    _check(run, GOLDEN["class"][cid]["full"], cid)
