"""K1 micro-benchmark on one MI355X: host vs device cost of a MulticlassAccuracy update.

Reports (bs=8192, C=1000, fp32 unless --dtype):
  * python_update_us   : MulticlassAccuracy.update() in a Python loop (what bench.py times)
  * raw_launch_us      : direct _C.cls_counts call in a loop (binding + launch only)
  * graph_us           : 100 updates captured in one HIP graph, replayed -> device time/update
  * eager_ref_us       : the reference's eager ATen chain (argmax/eq/long/sum/tensor/add)
  * grid sweep         : graph-timed device time per TORCHEVAL_AMD max_blocks setting
"""

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from torcheval_amd import _C
from torcheval_amd.metrics import MulticlassAccuracy


def timeit(fn, iters, warm=50):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e6


def graph_time(body, reps=100, replays=20):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            body(0)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for i in range(reps):
            body(i)
    g.replay()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(replays):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / (replays * reps) * 1e6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=8192)
    ap.add_argument("--c", type=int, default=1000)
    ap.add_argument("--dtype", default="float32")
    ap.add_argument("--pool", type=int, default=8)
    args = ap.parse_args()
    dt = getattr(torch, args.dtype)
    dev = torch.device("cuda")
    xs = [torch.randn(args.n, args.c, device=dev).to(dt) for _ in range(args.pool)]
    ys = [torch.randint(0, args.c, (args.n,), device=dev) for _ in range(args.pool)]
    res = {"n": args.n, "c": args.c, "dtype": args.dtype}

    m = MulticlassAccuracy(device=dev)
    i = [0]

    def upd():
        k = i[0] % args.pool
        i[0] += 1
        m.update(xs[k], ys[k])

    res["python_update_us"] = timeit(upd, 5000)
    xt, yt = xs[0][:64].contiguous(), ys[0][:64].contiguous()
    mt = MulticlassAccuracy(device=dev)
    res["host_only_update_us"] = timeit(lambda: mt.update(xt, yt), 5000)
    out = torch.zeros(2, device=dev)

    def raw():
        k = i[0] % args.pool
        i[0] += 1
        _C.cls_counts(xs[k], ys[k], 1, args.c, out[0:1], out[1:2], None, None, None, None, None, 0)

    res["raw_launch_us"] = timeit(raw, 5000)

    def body_for(blocks):
        def body(j):
            k = j % args.pool
            _C.cls_counts(xs[k], ys[k], 1, args.c, out[0:1], out[1:2], None, None, None, None, None, blocks)
        return body

    res["graph_us"] = graph_time(body_for(0))
    sweep = {}
    for blocks in (128, 256, 512, 1024, 2048, 4096):
        sweep[blocks] = graph_time(body_for(blocks))
    res["grid_sweep_us"] = sweep

    nc = torch.tensor(0.0, device=dev)
    nt = torch.tensor(0.0, device=dev)

    @torch.inference_mode()
    def eager():
        nonlocal nc, nt
        k = i[0] % args.pool
        i[0] += 1
        x, y = xs[k], ys[k]
        mask = (torch.argmax(x, dim=1) == y).long()
        nc += mask.sum()
        nt += torch.tensor(y.shape[0])

    res["eager_ref_us"] = timeit(eager, 2000)
    bytes_per = args.n * args.c * xs[0].element_size() + args.n * 8
    res["graph_GBps"] = bytes_per / (res["graph_us"] * 1e-6) / 1e9
    print(json.dumps(res))


if __name__ == "__main__":
    main()
