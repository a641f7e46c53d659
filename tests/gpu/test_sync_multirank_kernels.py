"""The ws > 1 arithmetic of the sync kernels (csrc/kernels/sync_reduce.hip) on a real GPU.

A 1-GPU box cannot host a multi-rank RCCL world (RCCL refuses two ranks on one device,
profiles/rccl_two_rank_one_gpu_r3.txt), so the kernels that only run when ws > 1 are driven
here with synthetic gathered buffers shaped exactly as the collectives leave them:

* ``seg_reduce_rows`` on [ws][row] rows (ws in {2, 3, 8}), every dtype x {sum, max, min},
  NaN / +-inf / bool, bit-equal to the ATen form ``state_buffer._reduce_rows_torch`` (the
  path gloo syncs take);
* ``snapshot_flags`` for every rank of an 8-rank world, the 8 snapshots summed as the f32 SUM
  all-reduce would, then ``merge_flag_slots`` = the elementwise max of the ranks' flags
  (including words >= 2^16);
* the whole state-buffer sync with 2 and 4 gloo ranks sharing cuda:0 (so the gathered rows
  are HBM tensors and the HIP reduction runs), bit-equal across ranks and to the generic
  engine.

Reference path being replaced: torcheval/metrics/toolkit.py:371-391.
"""

import pytest
import torch

from torcheval_amd.ops import native
from torcheval_amd.parallel import state_buffer as sbm
from torcheval_amd.utils.test_utils.dist_pool import run_distributed

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)
DTYPES = [torch.float32, torch.float16, torch.bfloat16, torch.float64, torch.int64, torch.int32,
          torch.uint8, torch.bool, torch.int8, torch.int16]
OPS = ["sum", "max", "min"]


def _fill(dtype, ws, n, g, op):
    if dtype == torch.bool:
        return torch.rand(ws, n, generator=g) < 0.3
    if dtype.is_floating_point:
        # dyadic values: every partial sum is exact, so the fold order cannot matter
        v = torch.randint(-8, 9, (ws, n), generator=g).to(torch.float64) / 4
        v[torch.rand(ws, n, generator=g) < 0.04] = float("nan")
        v[torch.rand(ws, n, generator=g) < 0.03] = float("inf")
        v[torch.rand(ws, n, generator=g) < 0.03] = float("-inf")
        return v.to(dtype)
    info = torch.iinfo(dtype)
    lo, hi = max(info.min, -(1 << 40)), min(info.max, 1 << 40)
    return torch.randint(lo, hi + 1, (ws, n), generator=g, dtype=torch.int64).to(dtype)  # sums wrap


def _layout(ws, g):
    """Rows of 30 segments (10 dtypes x 3 ops) at 16-B aligned offsets, filled per rank."""
    offs, counts, dts, ops, fills = [], [], [], [], []
    off = 0
    for dtype in DTYPES:
        es = torch.empty((), dtype=dtype).element_size()
        for op in OPS:
            n = int(torch.randint(1, 300, (1,), generator=g))
            offs.append(off)
            counts.append(n)
            dts.append(sbm._DT_CODE[dtype])
            ops.append(sbm._OP_CODE[op])
            fills.append(_fill(dtype, ws, n, g, op).contiguous().view(torch.uint8).view(ws, n * es))
            off += (n * es + 15) // 16 * 16
    row = off
    rows = torch.zeros(ws, row, dtype=torch.uint8)
    for o, f in zip(offs, fills):
        rows[:, o : o + f.shape[1]] = f
    return rows, row, (offs, counts, dts, ops)


def _canon(out, segs):
    """Per-segment typed views with NaN positions split out (NaN payloads may differ)."""
    inv = {v: k for k, v in sbm._DT_CODE.items()}
    res = []
    for o, n, d in zip(segs[0], segs[1], segs[2]):
        dtype = inv[d]
        es = torch.empty((), dtype=dtype).element_size()
        v = out[o : o + n * es].view(dtype)
        res.append(v)
    return res


@pytest.mark.parametrize("ws", [2, 3, 8])
def test_seg_reduce_rows_matches_aten(ws):
    g = torch.Generator().manual_seed(100 + ws)
    rows, row, segs = _layout(ws, g)
    want = torch.zeros(row, dtype=torch.uint8)
    sbm._reduce_rows_torch(rows, want, segs, ws)
    got = torch.full((row,), 0xAB, dtype=torch.uint8, device=DEV)
    native().seg_reduce_rows(rows.reshape(-1).to(DEV), got, ws, *segs)
    got = got.cpu()
    for i, (a, b) in enumerate(zip(_canon(got, segs), _canon(want, segs))):
        if a.dtype.is_floating_point:
            na, nb = torch.isnan(a), torch.isnan(b)
            assert torch.equal(na, nb), (i, a.dtype)
            a, b = a[~na], b[~nb]
            assert torch.equal(a.view(torch.uint8), b.view(torch.uint8)), (i, a.dtype)
        else:
            assert torch.equal(a, b), (i, a.dtype, segs[3][i])
    # padding bytes between segments are not touched by the kernel
    covered = torch.zeros(row, dtype=torch.bool)
    for o, n, d in zip(*segs[:3]):
        es = torch.empty((), dtype={v: k for k, v in sbm._DT_CODE.items()}[d]).element_size()
        covered[o : o + n * es] = True
    assert bool((got[~covered] == 0xAB).all())


def test_seg_reduce_rows_through_gathered_helper():
    """``_reduce_gathered`` (the engine's entry) picks the kernel for HBM rows."""
    ws = 8
    g = torch.Generator().manual_seed(9)
    rows, row, segs = _layout(ws, g)
    want = torch.zeros(row, dtype=torch.uint8)
    sbm._reduce_rows_torch(rows, want, segs, ws)
    got = sbm._reduce_gathered(rows.reshape(-1).to(DEV), segs, ws, row).cpu()
    for a, b in zip(_canon(got, segs), _canon(want, segs)):
        if a.dtype.is_floating_point:
            assert torch.equal(torch.isnan(a), torch.isnan(b))
            a, b = a[~torch.isnan(a)], b[~torch.isnan(b)]
        assert torch.equal(a, b)


@pytest.mark.parametrize("words", [1, 3, 7])
def test_snapshot_and_merge_flag_slots_ws8(words):
    ws = 8
    g = torch.Generator().manual_seed(words)
    nbytes = 16 * 1000
    specials = torch.tensor([0, 1, 0xFFFF, 0x10000, 0x12345678, 0x7FFFFFFF, 0xFFFE0001 & 0x7FFFFFFF], dtype=torch.int64)
    flags = specials[torch.randint(0, len(specials), (ws, words), generator=g)].to(torch.int32)
    srcs = [torch.randint(0, 256, (nbytes,), generator=g, dtype=torch.int64).to(torch.uint8) for _ in range(ws)]
    snaps = []
    for r in range(ws):
        dst = torch.full((nbytes + ws * words * 8,), 0xCD, dtype=torch.uint8, device=DEV)
        err = flags[r].to(DEV)
        native().snapshot_flags(srcs[r].to(DEV), dst, err, words, r, ws)
        dst = dst.cpu()
        assert torch.equal(dst[:nbytes], srcs[r])
        slots = dst[nbytes:].view(torch.float32).view(ws, words, 2)
        for q in range(ws):
            if q == r:
                u = flags[r].to(torch.int64) & 0xFFFFFFFF
                assert torch.equal(slots[q, :, 0], (u >> 16).to(torch.float32))
                assert torch.equal(slots[q, :, 1], (u & 0xFFFF).to(torch.float32))
            else:
                assert bool((slots[q] == 0).all())
        snaps.append(dst[nbytes:].view(torch.float32))
    summed = torch.stack(snaps).sum(0)  # what the f32 SUM all-reduce delivers (exact: one term each)
    merged = torch.full((words,), -1, dtype=torch.int32, device=DEV)
    native().merge_flag_slots(summed.to(DEV), merged, words, ws)
    assert torch.equal(merged.cpu(), flags.max(0).values)


def test_snapshot_flags_without_err_writes_zero_slots():
    ws, words = 4, 2
    src = torch.arange(64, dtype=torch.uint8, device=DEV)
    dst = torch.full((64 + ws * words * 8,), 7, dtype=torch.uint8, device=DEV)
    native().snapshot_flags(src, dst, None, words, 3, ws)
    assert torch.equal(dst[:64], src)
    assert bool((dst[64:].view(torch.float32) == 0).all())


def _gpu_fast_vs_general_job(rank, ws):
    """tests/metrics/test_rehearsal_collectives.py::_fast_vs_general_job on HBM states."""
    from torcheval_amd.metrics import Max, Mean, MulticlassAccuracy, MulticlassConfusionMatrix, MulticlassPrecision
    from torcheval_amd.parallel import state_buffer, state_sync

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    g = torch.Generator().manual_seed(10 + rank)

    def d(t):
        return t.to(dev)

    coll = {
        "acc": MulticlassAccuracy(num_classes=5, average="macro", device=dev).update(
            d(torch.randn(40, 5, generator=g)), d(torch.randint(0, 5, (40,), generator=g))),
        "micro": MulticlassAccuracy(device=dev).update(d(torch.randn(40, 5, generator=g)),
                                                       d(torch.randint(0, 5, (40,), generator=g))),
        "prec": MulticlassPrecision(num_classes=5, average=None, device=dev).update(
            d(torch.randn(40, 5, generator=g)), d(torch.randint(0, 5, (40,), generator=g))),
        "mean": Mean(device=dev).update(d(torch.randn(17, generator=g))),
        "max": Max(device=dev).update(d(torch.randn(9, generator=g))),
        "cm": MulticlassConfusionMatrix(200, device=dev).update(d(torch.randn(3000, 200, generator=g)),
                                                                d(torch.randint(0, 200, (3000,), generator=g))),
    }
    general = state_sync.start_sync_collection(coll, None, ws, snapshot=False, blocking=True).finish()
    fast = state_buffer.fast_sync(coll, None, ws)
    assert fast is not None
    single = state_buffer.fast_sync({"m": coll["micro"]}, None, ws)["m"]
    out = []
    for key in coll:
        for name in coll[key]._state_merge_kinds():
            a, c = getattr(fast[key], name), getattr(general[key], name)
            assert a.is_cuda, (key, name)
            assert torch.equal(a, c.to(a.device)), (key, name)
        out.append([float(x) for x in fast[key].compute().double().reshape(-1)[:50].cpu()])
    assert torch.equal(single.num_correct, fast["micro"].num_correct)
    # every rank's counts arrived: the synced total is the sum over ranks
    assert float(fast["micro"].num_total) == 40.0 * ws
    assert float(fast["cm"].confusion_matrix.sum()) == 3000.0 * ws
    return out


@pytest.mark.parametrize("ws", [2, 4])
def test_state_buffer_sync_gloo_ranks_on_one_gpu(ws):
    res = run_distributed(_gpu_fast_vs_general_job, ws, timeout=240.0)
    assert all(r == res[0] for r in res), "ranks disagree"
