"""Host cost of the direct RCCL primitives on a 1-rank group (us per call, back-to-back,
device-synchronised at the end): ncclAllGather vs ncclAllReduce (in place / out of place) of
8 bytes, against torch.distributed's all_gather_into_tensor / all_reduce and one ATen launch."""
import json
import os
import socket
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _t(fn, n=500):
    for _ in range(50):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return round((time.perf_counter() - t0) / n * 1e6, 2)


def main():
    from torcheval_amd.parallel import rccl_direct

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_port()}", rank=0, world_size=1, device_id=dev)
    h = rccl_direct.comm_for(dist.group.WORLD, 1, dev)
    src = torch.ones(2, device=dev)
    out = torch.empty(2, device=dev)
    res = {
        "direct_all_gather_8B": _t(lambda: rccl_direct.all_gather(h, src, out)),
        "direct_all_reduce_8B_inplace": _t(lambda: rccl_direct.all_reduce(h, out, "sum")),
        "direct_all_reduce_8B_out": _t(lambda: rccl_direct.all_reduce(h, src, "sum", out=out)),
        "torch_all_gather_into_tensor_8B": _t(lambda: dist.all_gather_into_tensor(out, src)),
        "torch_all_reduce_8B": _t(lambda: dist.all_reduce(out)),
        "aten_add_": _t(lambda: out.add_(1.0)),
        "empty_2": _t(lambda: torch.empty(2, device=dev)),
    }
    dist.destroy_process_group()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
