"""Frechet Inception Distance (parity: metrics/image/fid.py:53-274).

MI355X path:
* update: features from the model, then the K8 FP32-MFMA symmetric rank-k kernel adds
  act^T act (upper-triangle tiles, mirrored) and the column sums straight into the states -
  half the FLOPs of the reference's dense ``act.T @ act`` and no separate ``sum``.  On ROCm the
  activations are first staged in HBM (one copy per update, ``TORCHEVAL_AMD_FID_STAGE_ROWS``
  rows per side, 8192 by default = 64 MB at D = 2048) and K8 runs once per full stage (K =
  8192: ~44 ns per row against ~57 at K = 1000) or when a state is read (compute, sync,
  state_dict, copies), so the states always reflect every update;
* compute: tr sqrt(S1 S2) in FP64 from the symmetric L^T S2 L (S1 = L L^T, Cholesky) with an
  eigenvalues-only ``eigvalsh``, instead of the reference's non-symmetric ``linalg.eigvals``
  (better conditioned, identical in exact arithmetic).  On ROCm: one covariance pass per side
  (fid_prep.hip), the one-launch K9d Cholesky, the triangle-aware sandwich and the on-chip K9b
  eigenvalues; when both sides have fewer samples than features (singular covariances), the
  one-launch K9p pivoted Cholesky gives S1 = W^T W and K9b takes the r x r W S2 W^T;
* sync: every state is ``merge="sum"``, so syncing is one RCCL all-reduce of 2 x D^2 + 2 x D
  floats; the model itself is never pickled or transferred (the reference all-gathers the
  whole pickled metric, Inception-v3 included).
"""

import warnings
from typing import Any, Iterable, Optional, Union

import torch
from torch import nn, Tensor

from torcheval_amd.metrics.metric import Metric, inference_update
from torcheval_amd.models.inception import FIDInceptionV3
from torcheval_amd.ops import use_native
from torcheval_amd.ops.hostread import read_int

__all__ = ["FrechetInceptionDistance", "FIDInceptionV3"]


def _cov_update(act: Tensor, cov_sum: Tensor, col_sum: Tensor) -> None:
    if (
        use_native(act)
        and act.dtype == torch.float32
        and cov_sum.dtype == torch.float32
        and col_sum.dtype == torch.float32
        and act.dim() == 2
    ):
        from torcheval_amd.ops import native

        a = act
        # K8 stages 16-B row pieces: rows 16-B aligned (a width that is not a multiple of 4 is
        # zero-padded by the op itself when the tensor is contiguous)
        def _ok(t: Tensor) -> bool:
            return t.stride(1) == 1 and t.data_ptr() % 16 == 0 and (t.stride(0) % 4 == 0 or t.is_contiguous())

        if not _ok(a):
            # a fresh allocation: contiguous() would return a contiguous but misaligned view as is
            a = act.clone(memory_format=torch.contiguous_format)
        if _ok(a):
            native().fid_cov_update(a, cov_sum, col_sum)
            return
    col_sum += torch.sum(act, dim=0)
    cov_sum += torch.matmul(act.T, act)


def _tr_sqrt_product(s1: Tensor, s2: Tensor, n1: Optional[int] = None, n2: Optional[int] = None) -> Tensor:
    """tr sqrt(S1 S2) for symmetric PSD S1, S2 (FP64, both exactly symmetric): the sum of the
    square roots of ``_spectrum(s1, s2, n1, n2)``."""
    lam = _spectrum(s1, s2, n1, n2)
    return lam.clamp(min=0).sqrt().sum()


def _spectrum(s1: Tensor, s2: Tensor, n1: Optional[int] = None, n2: Optional[int] = None, finish=None) -> Tensor:
    """Eigenvalues (FP64) whose square roots sum to tr sqrt(S1 S2).

    The eigenvalues of S1 S2 equal those of the symmetric L^T S2 L when S1 = L L^T, so the
    fast path is one Cholesky (K9d), the triangle-aware sandwich and ONE eigenvalues-only
    ``eigvalsh`` (K9b; no eigenvectors, no back-transformation); on ROCm the three launch
    back to back and ONE host read checks both kernels' status words (``_spectrum_fast``).  A
    singular S1 (fewer samples than features) has no Cholesky factor; the same holds with the
    roles swapped when S2 has one.  When both are singular, S1 = W^T W with W [r, D] of rank r,
    and the eigvalsh runs on the r x r matrix W S2 W^T: the same non-zero spectrum as S1 S2.  On
    ROCm W comes from K9p (csrc/kernels/pivchol.hip), a pivoted (rank-revealing) Cholesky
    stopping at the LAPACK dpstrf tolerance D eps max diag; elsewhere (and as K9p's fallback)
    from ``eigh`` over the eigenvalues above the ``matrix_rank`` tolerance of the FP64 matrix.
    Both tolerances are the FP64 ones: covariances assembled from FP32 state sums carry
    rounding "noise" spectrum well above them, and the reference's ``eigvals(S1 S2)`` includes
    its square roots too, so it is kept (r is then the FP64 numerical rank, usually above the
    sample rank).

    ``n1`` / ``n2`` (optional sample counts) mark a side with n <= D as singular up front, so
    its Cholesky is not attempted; the pivoted factor then takes the side with fewer samples.

    ``finish`` (optional callable): applied to the returned eigenvalues, once they are final (the
    fast path applies it before its status read, see ``_spectrum_fast``)."""
    return _spectrum_checked(s1, s2, n1, n2, finish)


def _spectrum_checked(s1: Tensor, s2: Tensor, n1: Optional[int], n2: Optional[int], finish) -> Tensor:
    d = s1.shape[0]
    sing1 = n1 is not None and n1 <= d
    sing2 = n2 is not None and n2 <= d

    def done(lam: Tensor) -> Tensor:
        if finish is not None:
            finish(lam)
        return lam

    if not sing1:
        lam, info = _spectrum_fast(s1, s2, finish)
        if lam is not None:
            return lam  # finish already applied (speculatively, before the clean status read)
        if info is None:  # not applicable / a grid aborted: the checked sequence
            L, info = _chol(s1)
            if info == 0:
                return done(sym_eigvalsh(_lt_s_l(L, s2)))
    if not sing2:
        # S1 singular, S2 not: S1 S2 and S2 S1 share their spectrum, so factor S2 instead
        # (one more Cholesky rather than a rank-revealing factorisation)
        L2, info2 = _chol(s2)
        if info2 == 0:
            return done(sym_eigvalsh(_lt_s_l(L2, s1)))
    a, b = (s2, s1) if (n1 is not None and n2 is not None and n2 < n1) else (s1, s2)
    w = _pivoted_factor(a)
    if w is None:
        w = _eigh_factor(a)
    if w.shape[0] == 0:
        return done(torch.zeros(0, dtype=s1.dtype, device=s1.device))
    m = w @ (b @ w.T)
    return done(sym_eigvalsh((m + m.T) / 2))


def _spectrum_fast(s1: Tensor, s2: Tensor, finish=None) -> "tuple[Optional[Tensor], Optional[int]]":
    """K9d Cholesky -> triangle-aware sandwich -> K9b eigenvalues launched back to back with ONE
    host read of both kernels' status words (a host read after the Cholesky cost ~70 us of idle
    GPU, profiles/README.md round 6): (eigenvalues, 0), or (None, info != 0) when S1 is not
    positive definite, or (None, None) when the path does not apply or a grid aborted (the
    caller then takes the checked sequence).  ``finish`` (optional) is called on the eigenvalues
    BEFORE the status read, so the caller's closing launch is queued behind the eigensolver
    instead of after a host round trip (~45 us of idle GPU); when the status is bad the caller's
    later ``finish`` of the checked result overwrites it (stream order)."""
    n = s1.shape[0]
    if not (use_native(s1) and s1.dtype == torch.float64 and s1.dim() == 2 and 3 <= n <= 2560):
        return None, None
    from torcheval_amd.ops import native
    from torcheval_amd.ops.hostread import read_ints

    nat = native()
    nt = nat.cholesky_tiles(n)
    N = 64 * nt
    a = s1 if s1.stride(1) == 1 else s1.contiguous()
    L = torch.empty(N, N, dtype=torch.float64, device=s1.device)
    linv = torch.empty(nt * 4096, dtype=torch.float64, device=s1.device)
    ctl = torch.empty(1, dtype=torch.int32, device=s1.device)
    status = torch.zeros(3, dtype=torch.int32, device=s1.device)  # K9d info, abort; K9b status
    nat.cholesky_factor(a, L, linv, ctl, status[:2])
    m = _lt_s_l(L[:n, :n], s2).contiguous()
    lam = torch.empty(n, dtype=torch.float64, device=s1.device)
    if nat.sym_eigvals(m, lam, status[2:]) != 0:
        return None, None
    if finish is not None:
        finish(lam)  # speculative: valid when the status below is clean
    info, abort, eig = read_ints(status)
    if abort != 0:
        return None, None
    if info != 0:
        return None, info
    return (lam, 0) if eig == 0 else (None, None)


def _sqrt_eig_sum(m: Tensor) -> Tensor:
    return sym_eigvalsh(m).clamp(min=0).sqrt().sum()


def _eigh_factor(s: Tensor) -> Tensor:
    """W [r, D] with S = W^T W from ``eigh``: the eigenvectors of the eigenvalues above the FP64
    ``matrix_rank`` tolerance, scaled by their square roots (the CPU path and K9p's fallback)."""
    lam, vec = torch.linalg.eigh(s)
    keep = lam > lam.max().clamp(min=0) * lam.numel() * torch.finfo(lam.dtype).eps
    return (vec[:, keep] * lam[keep].sqrt()).T


def _pivoted_factor(s: Tensor) -> Optional[Tensor]:
    """W [r, D] with S = W^T W + O(tol) from K9p's pivoted Cholesky (rows in the original
    feature order), or None when the native path does not apply / its grid aborted."""
    n = s.shape[0]
    if not (use_native(s) and s.dtype == torch.float64 and s.dim() == 2 and 1 <= n <= 2048):
        return None
    from torcheval_amd.ops import native
    from torcheval_amd.ops.hostread import read_ints

    nat = native()
    N = nat.pivchol_padded(n)
    a = s if s.stride(1) == 1 else s.contiguous()
    slots = torch.empty(nat.pivchol_slot_words(n), dtype=torch.int64, device=s.device)
    w = torch.empty(N, N, dtype=torch.float64, device=s.device)
    piv = torch.empty(n, dtype=torch.int32, device=s.device)
    info = torch.empty(2, dtype=torch.int32, device=s.device)
    ctl = torch.empty(1, dtype=torch.int32, device=s.device)
    if nat.pivchol(a, slots, w, piv, info, ctl) != 0:
        return None  # (the grid could not be co-scheduled)
    rank, status = read_ints(info)
    if status & 2:
        warnings.warn("K9p pivoted Cholesky grid aborted (a hand-off timed out); using eigh", RuntimeWarning)
        return None
    if status & 1:  # a NaN in the matrix: the result is NaN, as the eigh path's would be
        return torch.full((1, n), float("nan"), dtype=torch.float64, device=s.device)
    return w[:rank, :n]


def _sandwich_blocks(n: int) -> int:
    # 2 block columns: 2.5 n^3 flops instead of the dense 4 n^3 in 4 library GEMMs, 0.41 ms at
    # D = 2048 against 0.54 for the two dense GEMMs; 3 / 4 / 8 blocks skip more zeros but their
    # narrow GEMMs run at half the rate: 0.51 / 0.55 / 0.83 ms (profiles/fid_compute_timing_r6.json).
    # TORCHEVAL_AMD_FID_SANDWICH_P: A/B of the block count (1 = the dense two GEMMs)
    import os

    p = int(os.environ.get("TORCHEVAL_AMD_FID_SANDWICH_P", "2"))
    return p if n >= 512 else 1


def _lt_s_l(L: Tensor, s: Tensor) -> Tensor:
    """L^T S L for lower-triangular L and symmetric S, exactly symmetric (FP64).

    On ROCm, triangle-aware: with L cut into p block columns, Y^T = L^T S is p GEMMs whose
    inner dimension skips L's zero blocks (block c: L[c0:, c]^T S[c0:, :]), and M = L^T Y is
    computed for its lower block triangle only (block row r: L[r0:, r]^T Y[r0:, :r1]) - 2.5 n^3
    instead of 4 n^3 flops at p = 2 - then ``sym_fill_upper`` mirrors the lower triangle (the
    diagonal blocks are computed whole)."""
    n = L.shape[0]
    p = _sandwich_blocks(n) if use_native(L) else 1
    if p == 1:
        m = L.T @ s @ L
        return (m + m.T) / 2
    from torcheval_amd.ops import native

    b = -(-n // p)
    b = -(-b // 64) * 64
    yt = torch.empty(n, n, dtype=L.dtype, device=L.device)
    for c0 in range(0, n, b):
        c1 = min(n, c0 + b)
        torch.mm(L[c0:, c0:c1].T, s[c0:, :], out=yt[c0:c1])
    m = torch.empty(n, n, dtype=L.dtype, device=L.device)
    for r0 in range(0, n, b):
        r1 = min(n, r0 + b)
        torch.mm(L[r0:, r0:r1].T, yt[:r1, r0:].T, out=m[r0:r1, :r1])
    native().sym_fill_upper(m)
    return m


def _chol(s: Tensor) -> "tuple[Tensor, int]":
    """(lower Cholesky factor, LAPACK info as a host int) of a symmetric FP64 matrix."""
    n = s.shape[0]
    if use_native(s) and s.dtype == torch.float64 and s.dim() == 2 and 1 <= n <= 16384:
        from torcheval_amd.ops import native
        from torcheval_amd.ops.hostread import read_ints

        nat = native()
        nt = nat.cholesky_tiles(n)
        N = 64 * nt
        a = s if s.stride(1) == 1 else s.contiguous()
        L = torch.empty(N, N, dtype=torch.float64, device=s.device)
        linv = torch.empty(nt * 4096, dtype=torch.float64, device=s.device)
        ctl = torch.empty(1, dtype=torch.int32, device=s.device)
        status = torch.empty(2, dtype=torch.int32, device=s.device)
        nat.cholesky_factor(a, L, linv, ctl, status)
        info, abort = read_ints(status)
        if not abort:
            return L[:n, :n], info
        warnings.warn("K9d Cholesky grid aborted (a hand-off timed out); using torch.linalg.cholesky_ex",
                      RuntimeWarning)
    L, info = torch.linalg.cholesky_ex(s)
    return L, int(info)


def cholesky_ex(s: Tensor) -> "tuple[Tensor, Tensor]":
    """Lower Cholesky factor of a symmetric FP64 matrix and an int ``info`` (0 = success, as
    ``torch.linalg.cholesky_ex``).

    On ROCm, K9d (``csrc/kernels/cholesky.hip``): the whole blocked factorisation in one
    persistent launch (64 x 64 tiles on FP64 MFMA, a dataflow of ticket-ordered tile tasks,
    one cross-CU hand-off per tile column) - instead of rocSOLVER's chain of ~160 us potf2
    launches and its trsm, or round 5's per-block launch loop."""
    L, info = _chol(s)
    return L, torch.tensor(info, dtype=torch.int32)


def sym_eigvalsh(m: Tensor) -> Tensor:
    """Eigenvalues (ascending) of a symmetric FP64 matrix.

    On ROCm, K9b (``csrc/kernels/symeig.hip``): the matrix stays on chip (the registers of one
    workgroup per CU) for the whole Householder reduction (one cooperative launch, one
    hand-off per column) and a multisection kernel finds the tridiagonal's eigenvalues - instead of rocSOLVER's
    ~7000 small launches.  Sizes the kernel does not take (n > 2560, n < 3), a grid the device
    cannot co-schedule, or an aborted grid fall back to ``torch.linalg.eigvalsh``."""
    if use_native(m) and m.dtype == torch.float64 and m.dim() == 2 and 3 <= m.shape[0] <= 2560:
        from torcheval_amd.ops import native

        mc = m.contiguous()
        lam = torch.empty(m.shape[0], dtype=torch.float64, device=m.device)
        status = torch.zeros(1, dtype=torch.int32, device=m.device)
        if native().sym_eigvals(mc, lam, status) == 0 and read_int(status) == 0:
            return lam
    return torch.linalg.eigvalsh(m)


def frechet_distance(mu1: Tensor, sigma1: Tensor, mu2: Tensor, sigma2: Tensor) -> Tensor:
    """||mu1 - mu2||^2 + tr S1 + tr S2 - 2 tr sqrt(S1 S2)  (FP64, symmetric formulation)."""
    s1 = sigma1.double()
    s2 = sigma2.double()
    return _frechet_symmetric(mu1, (s1 + s1.T) / 2, mu2, (s2 + s2.T) / 2)


def _frechet_symmetric(mu1: Tensor, s1: Tensor, mu2: Tensor, s2: Tensor, n1: Optional[int] = None,
                       n2: Optional[int] = None) -> Tensor:
    """``frechet_distance`` of exactly symmetric FP64 covariances (``n1`` / ``n2``: sample
    counts, see ``_tr_sqrt_product``)."""
    mu1, mu2 = mu1.double(), mu2.double()
    tr_sqrt = _tr_sqrt_product(s1, s2, n1, n2)
    return (mu1 - mu2).square().sum() + s1.trace() + s2.trace() - 2 * tr_sqrt


def _covariance(cov_sum: Tensor, col_sum: Tensor, n: int) -> Tensor:
    """The exactly symmetric FP64 covariance (C / 2 + C^T / 2 - n mu mu^T) / (n - 1) from the
    states (reference fid.py:239-250 forms it with the outer product in the states' dtype).
    On ROCm one ``cov_finalize`` pass (csrc/kernels/fid_prep.hip) instead of ~10 FP64 passes."""
    if (use_native(cov_sum) and cov_sum.dtype == torch.float32 and col_sum.dtype == torch.float32
            and cov_sum.is_contiguous() and col_sum.is_contiguous() and n > 1):
        from torcheval_amd.ops import native

        out = torch.empty(cov_sum.shape, dtype=torch.float64, device=cov_sum.device)
        native().cov_finalize(cov_sum, col_sum, float(n), out)
        return out
    mean = col_sum.double() / n
    c = (cov_sum.double() - n * torch.outer(mean, mean)) / (n - 1)
    return (c + c.T) / 2


_STATES = (("real_sum", "real_cov_sum", "num_real_images"), ("fake_sum", "fake_cov_sum", "num_fake_images"))


def _staged_state(name: str, side: int) -> property:
    """A state whose value folds the side's staged activations in before it is read; assigning
    it (load_state_dict, reset, sync results) drops the side's staged rows with the old value."""
    key = "_" + name

    def get(self):
        d = self.__dict__
        rows = d.get("_stage_rows")
        if rows is not None and rows[side]:
            self._flush(side)
        return d[key]

    def set(self, value):
        d = self.__dict__
        rows = d.get("_stage_rows")
        if rows is not None:
            rows[side] = 0
        d[key] = value

    return property(get, set)


def _stageable(act: Tensor) -> bool:
    """Stage on the native (ROCm) path, where K8's per-launch cost is what staging amortises."""
    return use_native(act)


def _stage_rows_default() -> int:
    import os

    return max(int(os.environ.get("TORCHEVAL_AMD_FID_STAGE_ROWS", "8192")), 0)


class FrechetInceptionDistance(Metric[torch.Tensor]):
    """
    FID between real and generated images.

    Args:
        model: feature extractor mapping images to [B, feature_dim] activations; default the
            native Inception-v3 (``FIDInceptionV3``, random weights unless a local checkpoint
            is supplied - see ``torcheval_amd.models.inception``).
        feature_dim: activation width (2048 for the default model).
    """

    def __init__(
        self,
        model: Optional[nn.Module] = None,
        feature_dim: int = 2048,
        device: Optional[torch.device] = None,
    ) -> None:
        super().__init__(device=device)
        self._FID_parameter_check(model=model, feature_dim=feature_dim)
        if model is None:
            model = FIDInceptionV3()
        self.model = model.to(self.device)
        self.model.eval()
        d = feature_dim
        self._feature_dim = d
        self._stage = [None, None]  # per side: [rows, D] float32 HBM staging buffer (ROCm)
        self._stage_rows = [0, 0]
        self._add_state("real_sum", torch.zeros(d, device=self.device), merge="sum")
        self._add_state("real_cov_sum", torch.zeros((d, d), device=self.device), merge="sum")
        self._add_state("fake_sum", torch.zeros(d, device=self.device), merge="sum")
        self._add_state("fake_cov_sum", torch.zeros((d, d), device=self.device), merge="sum")
        self._add_state("num_real_images", torch.tensor(0, device=self.device).int(), merge="sum")
        self._add_state("num_fake_images", torch.tensor(0, device=self.device).int(), merge="sum")

    @inference_update
    def update(self, images: Tensor, is_real: bool) -> "FrechetInceptionDistance":
        """Add a batch of [B, 3, H, W] images (float32 in [0, 1] for the default model)."""
        self._FID_update_input_check(images=images, is_real=is_real)
        images = images.to(self.device)
        activations = self.model(images)
        return self.update_activations(activations, is_real)

    @torch.inference_mode()
    def update_activations(self, activations: Tensor, is_real: bool) -> "FrechetInceptionDistance":
        """Add precomputed [B, feature_dim] activations (skips the feature extractor)."""
        activations = activations.to(self.device)
        b = activations.shape[0]
        side = 0 if is_real else 1
        cap = _stage_rows_default()
        if (0 < b <= cap and _stageable(activations) and activations.dtype == torch.float32
                and activations.dim() == 2 and activations.shape[1] == self._feature_dim):
            d = self.__dict__
            stage = d["_stage"][side]
            if d["_stage_rows"][side] + b > cap or (stage is not None and (
                    stage.shape[0] != cap or stage.device != activations.device)):
                self._flush(side)
            if stage is None or stage.shape[0] != cap or stage.device != activations.device:
                stage = d["_stage"][side] = torch.empty(cap, self._feature_dim, dtype=torch.float32,
                                                        device=activations.device)
            r = d["_stage_rows"][side]
            stage[r : r + b].copy_(activations)  # one copy now; K8 runs once per full stage
            d["_stage_rows"][side] = r + b
            return self
        names = _STATES[side]
        setattr(self, names[2], getattr(self, names[2]) + b)
        _cov_update(activations, getattr(self, names[1]), getattr(self, names[0]))
        return self

    def _flush(self, side: int) -> None:
        """Fold the side's staged activations into its states: ONE K8 launch over all staged
        rows (column sums fused) and one count update."""
        d = self.__dict__
        rows = d["_stage_rows"][side]
        if not rows:
            return
        d["_stage_rows"][side] = 0
        s, cov, n = ("_" + name for name in _STATES[side])
        with torch.inference_mode():
            _cov_update(d["_stage"][side][:rows], d[cov], d[s])
            d[n] += rows

    def __getstate__(self):
        # copies (copy / deepcopy / pickle) carry folded states and no staging buffers
        for side in (0, 1):
            self._flush(side)
        state = dict(self.__dict__)
        state["_stage"] = [None, None]
        state["_stage_rows"] = [0, 0]
        return state

    def __setstate__(self, state) -> None:
        self.__dict__.update(state)

    def reset(self) -> "FrechetInceptionDistance":
        self.__dict__["_stage_rows"] = [0, 0]  # staged rows belong to the values being reset
        return super().reset()

    @torch.inference_mode()
    def merge_state(self, metrics: Iterable["FrechetInceptionDistance"]) -> "FrechetInceptionDistance":
        for metric in metrics:
            self.real_sum += metric.real_sum.to(self.device)
            self.real_cov_sum += metric.real_cov_sum.to(self.device)
            self.fake_sum += metric.fake_sum.to(self.device)
            self.fake_cov_sum += metric.fake_cov_sum.to(self.device)
            self.num_real_images += metric.num_real_images.to(self.device)
            self.num_fake_images += metric.num_fake_images.to(self.device)
        return self

    @torch.inference_mode()
    def compute(self) -> Tensor:
        from torcheval_amd.ops.hostread import read_int_pair

        # both counts in one host read (one publish launch; stacking them first cost three small
        # launches ahead of the read)
        nr, nf = read_int_pair(self.num_real_images, self.num_fake_images)
        if nr == 0 or nf == 0:
            warnings.warn(
                "Computing FID requires at least 1 real image and 1 fake image,"
                f"but currently running with {nr} real images and {nf} fake images."
                "Returning 0.0",
                RuntimeWarning,
            )
            return torch.tensor(0.0)
        real_cov = _covariance(self.real_cov_sum, self.real_sum, nr)
        fake_cov = _covariance(self.fake_cov_sum, self.fake_sum, nf)
        if (use_native(real_cov) and self.real_sum.dtype == torch.float32 and self.fake_sum.dtype == torch.float32
                and real_cov.dtype == torch.float64 and fake_cov.dtype == torch.float64):
            # the spectrum, then ONE launch for |mu1 - mu2|^2 + tr S1 + tr S2 - 2 sum sqrt(lam)
            from torcheval_amd.ops import native

            out = torch.empty((), dtype=torch.float32, device=real_cov.device)
            rs, fs = self.real_sum.contiguous(), self.fake_sum.contiguous()

            def finish(lam: Tensor) -> None:
                native().fid_finish(rs, float(nr), fs, float(nf), real_cov, fake_cov, lam.contiguous(), out)

            _spectrum(real_cov, fake_cov, nr, nf, finish)
            return out
        real_mean = self.real_sum.double() / nr
        fake_mean = self.fake_sum.double() / nf
        return _frechet_symmetric(real_mean, real_cov, fake_mean, fake_cov, nr, nf).to(torch.float32)

    real_sum = _staged_state("real_sum", 0)
    real_cov_sum = _staged_state("real_cov_sum", 0)
    num_real_images = _staged_state("num_real_images", 0)
    fake_sum = _staged_state("fake_sum", 1)
    fake_cov_sum = _staged_state("fake_cov_sum", 1)
    num_fake_images = _staged_state("num_fake_images", 1)

    def _calculate_frechet_distance(self, mu1: Tensor, sigma1: Tensor, mu2: Tensor, sigma2: Tensor) -> Tensor:
        return frechet_distance(mu1, sigma1, mu2, sigma2)

    def _FID_parameter_check(self, model: Optional[nn.Module], feature_dim: int) -> None:
        if feature_dim is None or feature_dim <= 0:
            raise RuntimeError("feature_dim has to be a positive integer")
        if model is None and feature_dim != 2048:
            raise RuntimeError(
                "When the default Inception v3 model is used, feature_dim needs to be set to 2048"
            )

    def _FID_update_input_check(self, images: Tensor, is_real: bool) -> None:
        if not torch.is_tensor(images):
            raise ValueError(f"Expected tensor as input, but got {type(images)}.")
        if images.dim() != 4:
            raise ValueError(f"Expected 4D tensor as input. But input has {images.dim()} dimenstions.")
        if images.size()[1] != 3:
            raise ValueError(f"Expected 3 channels as input. Got {images.size()[1]}.")
        if type(is_real) != bool:
            raise ValueError(f"Expected 'real' to be of type bool but got {type(is_real)}.")
        if isinstance(self.model, FIDInceptionV3):
            if images.dtype != torch.float32:
                raise ValueError(
                    "When default inception-v3 model is used, images expected to be `torch.float32`, "
                    f"but got {images.dtype}."
                )
            if images.min() < 0 or images.max() > 1:
                raise ValueError(
                    "When default inception-v3 model is used, images are expected to be in the [0, 1] interval"
                )

    def to(self, device: Union[str, torch.device], *args: Any, **kwargs: Any) -> "FrechetInceptionDistance":
        super().to(device, *args, **kwargs)  # reading the states folds the staged rows in
        self.__dict__["_stage"] = [None, None]
        self.model.to(self.device)
        return self
