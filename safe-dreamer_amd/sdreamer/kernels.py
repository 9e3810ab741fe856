"""Typed wrappers over the C ABI (include/sdhip.h): shape checks in Python, launches on torch's current stream.

Raw kernel calls only (no autograd; that lives in sdreamer/ops.py). Every wrapper requires HIP device tensors:
there is no CPU fallback anywhere in the product path.
"""
from __future__ import annotations

import ctypes
import os

import torch

from . import _native as nat

EPS = 1e-4  # nn.RMSNorm(eps=1e-04) everywhere in the reference


def stream():
    return torch.cuda.current_stream().cuda_stream


def p(t):
    return 0 if t is None else t.data_ptr()


def _chk(*ts):
    for t in ts:
        if t is None:
            continue
        if not t.is_cuda:
            raise TypeError("sdreamer kernels need HIP device tensors (no CPU fallback)")


def _c(t):
    if not t.is_contiguous():
        raise ValueError("expected a contiguous tensor")
    return t


def empty(*shape, like=None, device=None, dtype=torch.float32):
    return torch.empty(*shape, dtype=dtype, device=device if device is not None else like.device)


# ------------------------------------------------------------------------------------------------- GEMM
def _layout(t, rows_dim, k_dim):
    sr, sk = t.stride(rows_dim), t.stride(k_dim)
    if sk == 1 and (t.shape[rows_dim] == 1 or sr >= t.shape[k_dim]):
        return True, max(sr, 1)
    if sr == 1:
        return False, max(sk, 1)
    if sk == 1:
        return True, max(sr, 1)
    raise ValueError(f"GEMM operand needs a unit stride, got strides {t.stride()} shape {tuple(t.shape)}")


def _skinny_split(M, N, K, batch):
    """K split for the skinny kernels: single launch when there are enough column tiles, else up to ~64 WGs."""
    if M <= 16:
        tiles = -(-N // 16) * batch
        if tiles >= 16 or K < 1024:
            return 1
        return max(1, min(-(-64 // tiles), K // 512))
    tiles = -(-N // 32) * batch
    ks = min(max(K // 128, 1), max(1, -(-256 // tiles)))
    return max(1, min(ks, 64))


# SDREAMER_F32_SPLIT2=1 (A/B knob): exact-f32 GEMMs of one round of 64 x 64 tiles (256..511) with K >= 1024 split K in
# two (the world-model phase's 1024 x 1024 x 1024 Barlow contractions: 256 workgroups over 32 k tiles each)
_F32_SPLIT2 = os.environ.get("SDREAMER_F32_SPLIT2", "0") == "1"


def _auto_split(M, N, K, batch):
    tiles = -(-M // 64) * -(-N // 64) * batch
    if _F32_SPLIT2 and 256 <= tiles < 512 and K >= 1024:
        return 2
    if tiles >= 256 or K < 512:
        return 1
    ks = min(K // 256, max(1, 512 // tiles))
    return max(1, min(ks, 32))


# SDREAMER_FAST_GEMM=0 keeps every contraction on the exact f32 MFMA path (A/B and precision studies)
FAST_GEMM = os.environ.get("SDREAMER_FAST_GEMM", "1") != "0"


# workgroups a long-K split-bf16 GEMM aims for: 512 (2 per CU). Alone the 256 x 2560 x 15360 weight gradient runs
# faster with more (1024: 157 vs 192 us), but in the update, beside the latency-bound scan backward, 512 measured
# best (11.70 vs 11.80 ms at 1024, 11.76 at 2048 per update; gpurun_out r04v); again in round 5 against fewer
# (10.70 vs 10.74 at 384, 10.86 at 256; profiles/r05wg)
_G3_WG_TARGET = int(os.environ.get("SDREAMER_G3_WGS", "512"))
# longest K chunk (rows) a split-bf16 workgroup takes when that needs more splits than the workgroup target — at most
# twice as many (SDREAMER_G3_CHUNK, off). The atari-like config's 256 x 3072 x 30720 weight gradients go from 10
# splits to 20 with 1536: 18.89 / 18.98 / 19.00 vs 18.89 / 18.89 / 18.85 ms per update, memory maze 74.30 vs 74.15
# (gpurun_out r04c) — no gain.
_G3_CHUNK = int(os.environ.get("SDREAMER_G3_CHUNK", "0"))


def _fast_split(M, N, K, batch):
    """K split for the split-bf16 kernel: ~_G3_WG_TARGET workgroups of 128x128 tiles when K is long, preferring a
    split that cuts K into equal whole 32-deep tiles; the launcher falls back to 64x64 tiles below 256 workgroups.
    (The 256 x 2560 x 15360 weight gradient alone: 13 splits 192 us, 20 157 us, 30 155 us, 60 186 us —
    tools/wgrad_sweep.py.)"""
    tiles = -(-M // 128) * -(-N // 128) * batch
    if tiles >= 256:
        return 1
    if K >= 1024:
        wg = -(-_G3_WG_TARGET // tiles)
        if _G3_CHUNK > 0:
            wg = max(wg, min(-(-K // _G3_CHUNK), 2 * wg))
        cap = max(1, min(K // 512, wg, 32))
        if K % 32 == 0:
            kt = K // 32
            even = [d for d in range(cap, 0, -1) if kt % d == 0]
            if even and even[0] * 2 > cap:
                return even[0]
        return cap
    # short K (e.g. the replay-value head on ~1k rows): 64x64 tiles, split so the launch still has ~256 workgroups
    t64 = -(-M // 64) * -(-N // 64) * batch
    if t64 >= 128 or K < 256:
        return 1
    return max(1, min(K // 128, -(-256 // t64), 16))


_WGRAD_T128 = int(os.environ.get("SDREAMER_WGRAD_T128", "0"))


def _wgrad_t128_split(M, N, K):
    """split count for ~_WGRAD_T128 workgroups of 128 x 128 tiles, an even divisor of K's 32-deep tiles if one is near"""
    tiles = -(-M // 128) * -(-N // 128)
    want = max(1, min(32, round(_WGRAD_T128 / tiles), K // 512))
    kt = K // 32 if K % 32 == 0 else 0
    if kt:
        for d in sorted(range(1, 33), key=lambda d: (abs(d - want), -d)):
            if kt % d == 0 and abs(d - want) <= max(1, want // 4):
                return d
    return want


def gemm(a, b, out, bias=None, alpha=1.0, beta=0.0, ksplit=None, tile=-1, fast=False, rowsum=None):
    """out[M,N] = alpha * a[M,K] @ b[K,N] (+ bias[N]) (+ beta*out). Strided views allowed (one unit stride each);
    3-D operands are a strided batch over dim 0. fast=True: split-bf16 MFMA path (sd_gemm_bf16x3, ~1e-5 relative)
    for contractions no sampled index depends on (gradients, frozen heads). rowsum (M,): also accumulate
    alpha * a's row sums into it in the same launch (sd_gemm_bf16x3_wgrad: a weight gradient's bias gradient);
    returns False without launching when that fused form does not apply (the caller reduces separately)."""
    _chk(a, b, out, bias)
    if a.dtype != torch.float32 or b.dtype != torch.float32 or out.dtype != torch.float32:
        raise TypeError("fp32 GEMM")
    if a.dim() == 3:
        Bt, M, K = a.shape
        Nn = b.shape[2]
        if b.shape[0] != Bt or b.shape[1] != K or tuple(out.shape) != (Bt, M, Nn):
            raise ValueError(f"gemm shapes {tuple(a.shape)} {tuple(b.shape)} {tuple(out.shape)}")
        ak, lda = _layout(a, 1, 2)
        bk, ldb = _layout(b, 2, 1)
        sA, sB, sC = a.stride(0), b.stride(0), out.stride(0)
        if out.stride(2) != 1:
            raise ValueError("gemm output needs unit column stride")
        ldc = out.stride(1)
        sBias = bias.stride(0) if (bias is not None and bias.dim() == 2) else 0
    else:
        Bt = 1
        M, K = a.shape
        Nn = b.shape[1]
        if b.shape[0] != K or tuple(out.shape) != (M, Nn):
            raise ValueError(f"gemm shapes {tuple(a.shape)} {tuple(b.shape)} {tuple(out.shape)}")
        ak, lda = _layout(a, 0, 1)
        bk, ldb = _layout(b, 1, 0)
        sA = sB = sC = sBias = 0
        if out.stride(1) != 1 and Nn > 1:
            raise ValueError("gemm output needs unit column stride")
        ldc = out.stride(0) if M > 1 else max(Nn, 1)
    if M == 0 or Nn == 0:
        return out
    fast = fast and FAST_GEMM and M >= 64 and Nn >= 64 and K >= 64
    if rowsum is not None and not (fast and Bt == 1 and not ak and rowsum.is_contiguous()):
        return False
    if ksplit is None and fast and _WGRAD_T128 and not ak and not bk and M <= 512 and K >= 4096 and tile < 0:
        # weight-gradient shape (dW = dy^T x: long K, both operands rows-contiguous) on 128 x 128 tiles with about
        # _WGRAD_T128 workgroups (SDREAMER_WGRAD_T128, A/B knob): fewer, longer split-K workgroups
        ksplit, tile = _wgrad_t128_split(M, Nn, K), 0
    if ksplit is None:
        if fast:
            ksplit = _fast_split(M, Nn, K, Bt)
        else:
            ksplit = _skinny_split(M, Nn, K, Bt) if (M <= 32 and ak and tile < 0) else _auto_split(M, Nn, K, Bt)
    d = nat.GemmDesc()
    d.A, d.B, d.C, d.bias = p(a), p(b), p(out), (p(bias) if bias is not None else None)
    d.lda, d.ldb, d.ldc = lda, ldb, ldc
    d.strideA, d.strideB, d.strideC, d.strideBias = sA, sB, sC, sBias
    d.M, d.N, d.K, d.batch = M, Nn, K, Bt
    d.a_kcontig, d.b_kcontig = int(ak), int(bk)
    d.ksplit, d.tile = int(ksplit), int(tile)
    d.alpha, d.beta = float(alpha), float(beta)
    ws = None
    if ksplit > 1:
        extra = ksplit * M if rowsum is not None else 0
        ws = torch.empty(ksplit * Bt * M * Nn + extra, dtype=torch.float32, device=out.device)
    if rowsum is not None:
        return nat.call_shaped("sd_gemm_bf16x3_wgrad", ctypes.byref(d), p(ws), ws.numel() if ws is not None else 0,
                               p(rowsum), 1, stream())
    nat.call("sd_gemm_bf16x3" if fast else "sd_gemm_f32", ctypes.byref(d), p(ws), ws.numel() if ws is not None else 0,
             stream())
    return out


def wgrad2(dy, x, dw, db_a, db_b, split):
    """Two linear layers' weight gradients over one input x in one split-bf16 GEMM: dw (Oa + Ob, I) += dy^T x with
    dy (R, Oa + Ob) their joint output gradient and dw a view over both weight gradients back to back; the bias
    gradients of rows < split go to db_a, the rest to db_b (sd_gemm_bf16x3_wgrad2). Returns False (nothing launched)
    for shapes outside the split-bf16 kernel (M, N or K < 64): the caller then runs per-layer wgrad()."""
    a = dy.t()
    M, Kk = a.shape
    Nn = x.shape[1]
    _chk(a, x, dw, db_a, db_b)
    if not (dw.is_contiguous() and db_a.is_contiguous() and db_b.is_contiguous() and tuple(dw.shape) == (M, Nn)
            and x.shape[0] == Kk and 0 < split < M and db_a.numel() == split and db_b.numel() == M - split):
        raise ValueError(f"wgrad2 shapes dy {tuple(dy.shape)} x {tuple(x.shape)} dw {tuple(dw.shape)} split {split}")
    ak, lda = _layout(a, 0, 1)
    bk, ldb = _layout(x, 1, 0)
    ksplit = _fast_split(M, Nn, Kk, 1)
    d = nat.GemmDesc()
    d.A, d.B, d.C, d.bias = p(a), p(x), p(dw), None
    d.lda, d.ldb, d.ldc = lda, ldb, Nn
    d.strideA = d.strideB = d.strideC = d.strideBias = 0
    d.M, d.N, d.K, d.batch = M, Nn, Kk, 1
    d.a_kcontig, d.b_kcontig = int(ak), int(bk)
    d.ksplit, d.tile = int(ksplit), -1
    d.alpha, d.beta = 1.0, 1.0
    ws = torch.empty(ksplit * M * Nn + ksplit * M, dtype=torch.float32, device=dw.device) if ksplit > 1 else None
    return nat.call_shaped("sd_gemm_bf16x3_wgrad2", ctypes.byref(d), p(ws), ws.numel() if ws is not None else 0,
                           p(db_a), p(db_b), int(split), 1, stream())


def wgrad(dy, x, dw, db=None):
    """nn.Linear backward's parameter gradients on the split-bf16 path: dw += dy^T x, db += column sums of dy (in the
    same launch when the shape allows, else a separate column-sum launch). dy (R, O), x (R, I), dw (O, I)."""
    if db is not None and gemm(dy.t(), x, dw, beta=1.0, fast=True, rowsum=db) is not False:
        return
    gemm(dy.t(), x, dw, beta=1.0, fast=True)
    if db is not None:
        colsum(dy, db, accumulate=True)


def mlp_layer(x, w, out, bias=None, norm_w=None, part_in=None, part_out=None, act=1, alpha=1.0):
    """One Linear of an MLP on the split-bf16 core with the previous layer's RMSNorm + SiLU fused into the A loader
    (sd_gemm_bf16x3_mlp): out[b] = act(rms(x[b]) * norm_w[b]) @ w[b]^T + bias[b]. Batched over dim 0 of 3-D operands
    (x may be an expanded (stride-0) view); norm_w None = x taken as is; part_in (n, q, M): the producer's row
    partial sums of squares; part_out (n, N / 64, M) receives this layer's. Returns False when the shape is outside the
    fused kernel (the caller then takes the unfused path).
    Per-entry form: w (and bias / norm_w) a list of n tensors, entry b's weight (N_b <= out.shape[2], K) row-major
    and contiguous: several heads' layers in one launch without stacking or zero-padding their weights (columns
    >= N_b of out[b] get 0)."""
    if isinstance(w, (list, tuple)):
        return _mlp_layer_entries(x, list(w), out, bias, norm_w, part_in, part_out, act, alpha)
    if x.dim() == 2:
        x, w, out = x[None], w[None], out[None]
        bias = bias[None] if bias is not None else None
        norm_w = norm_w[None] if norm_w is not None else None
        part_in = part_in[None] if part_in is not None else None
        part_out = part_out[None] if part_out is not None else None
    n, M, Kk = x.shape
    Nn = w.shape[1]
    _chk(x, w, out, bias)
    if x.stride(2) != 1 or w.stride(2) != 1 or not out.is_contiguous() or (bias is not None and bias.stride(1) != 1):
        return False
    d = nat.GemmDesc()
    d.A, d.B, d.C, d.bias = p(x), p(w), p(out), (p(bias) if bias is not None else None)
    d.lda, d.ldb, d.ldc = x.stride(1), w.stride(1), Nn
    d.strideA, d.strideB, d.strideC = x.stride(0), w.stride(0), M * Nn
    d.strideBias = bias.stride(0) if bias is not None else 0
    d.M, d.N, d.K, d.batch = M, Nn, Kk, n
    d.a_kcontig, d.b_kcontig, d.ksplit, d.tile = 1, 1, 1, 0
    d.alpha, d.beta = float(alpha), 0.0
    e = nat.MlpExt()
    if norm_w is not None:
        e.norm_w, e.stride_norm_w = p(norm_w), norm_w.stride(0)
        e.part_in, e.stride_part_in, e.npart_in = p(part_in), part_in.stride(0), part_in.shape[1]
        e.act, e.eps = int(act), EPS
    if part_out is not None:
        e.part_out, e.stride_part_out = p(part_out), part_out.stride(0)
    # byref (not addressof): a LaunchProbe's recorded arguments keep the extension struct alive for its replays
    return nat.call_shaped("sd_gemm_bf16x3_mlp", ctypes.byref(d), ctypes.byref(e), stream())


_MLP_MAXB = nat._define(nat.HEADER, "SD_MLP_MAXB")


def _mlp_layer_entries(x, ws, out, biases, norm_ws, part_in, part_out, act, alpha):
    n, M, Kk = x.shape
    Nn = out.shape[2]
    if n != len(ws) or n > _MLP_MAXB or tuple(out.shape[:2]) != (n, M):
        return False
    _chk(x, out, *ws)
    if x.stride(2) != 1 or not out.is_contiguous():
        return False
    for t in ws + list(biases or []) + list(norm_ws or []):
        if t.dtype != torch.float32 or not t.is_contiguous():
            return False
    if any(w.shape[1] != Kk or w.shape[0] > Nn for w in ws):
        raise ValueError(f"per-entry weights {[tuple(w.shape) for w in ws]} for K {Kk}, N {Nn}")
    d = nat.GemmDesc()
    d.A, d.B, d.C, d.bias = p(x), p(ws[0]), p(out), None
    d.lda, d.ldb, d.ldc = x.stride(1), Kk, Nn
    d.strideA, d.strideB, d.strideC, d.strideBias = x.stride(0), 0, M * Nn, 0
    d.M, d.N, d.K, d.batch = M, Nn, Kk, n
    d.a_kcontig, d.b_kcontig, d.ksplit, d.tile = 1, 1, 1, 0
    d.alpha, d.beta = float(alpha), 0.0
    e = nat.MlpExt()
    for b, w in enumerate(ws):
        e.w_ptr[b] = p(w)
        e.w_rows[b] = w.shape[0] if w.shape[0] < Nn else 0
        if biases is not None:
            e.bias_ptr[b] = p(biases[b])
        if norm_ws is not None:
            e.norm_w_ptr[b] = p(norm_ws[b])
    if norm_ws is not None:
        e.part_in, e.stride_part_in, e.npart_in = p(part_in), part_in.stride(0), part_in.shape[1]
        e.act, e.eps = int(act), EPS
    if part_out is not None:
        e.part_out, e.stride_part_out = p(part_out), part_out.stride(0)
    # byref (not addressof): a LaunchProbe's recorded arguments keep the extension struct alive for its replays
    return nat.call_shaped("sd_gemm_bf16x3_mlp", ctypes.byref(d), ctypes.byref(e), stream())


def mm(a, b, bias=None, out=None, **kw):
    M, Nn = a.shape[-2], b.shape[-1]
    if out is None:
        shape = (a.shape[0], M, Nn) if a.dim() == 3 else (M, Nn)
        out = torch.empty(shape, dtype=torch.float32, device=a.device)
    return gemm(a, b, out, bias=bias, **kw)


def linear(x, w, b=None, out=None, beta=0.0, fast=False):
    """x (M, I) @ w(O, I)^T + b  — nn.Linear forward."""
    return mm(x, w.t(), bias=b, out=out, beta=beta, fast=fast)


# ------------------------------------------------------------------------------------------------- row norms
def rmsnorm_fwd(x, w, act=1, y=None, rstd=None):
    """y may be a column slice of a wider row-major tensor (unit column stride)."""
    x = _c(x)
    N = x.shape[-1]
    M = x.numel() // N
    y = torch.empty_like(x) if y is None else y
    rstd = torch.empty(x.shape[:-1], dtype=torch.float32, device=x.device) if rstd is None else rstd
    if y.is_contiguous():
        nat.call("sd_rmsnorm_fwd", p(x), p(w), p(y), p(rstd), M, N, EPS, int(act), stream())
    else:
        if y.dim() != 2 or y.stride(1) != 1:
            raise ValueError("strided rmsnorm output must be a 2-D row-major slice")
        nat.call("sd_rmsnorm_fwd_ld", p(x), p(w), p(y), y.stride(0), p(rstd), M, N, EPS, int(act), stream())
    return y, rstd


def rmsnorm_bwd(x, w, rstd, dy, act=1, dx=None, dw=None, accumulate_dx=False, accumulate_dw=True):
    N = x.shape[-1]
    M = x.numel() // N
    if dy.dim() == 2 and dy.shape[1] == N and dy.stride(1) == 1 and not dy.is_contiguous():
        ldy = dy.stride(0)  # a column block of a wider gradient, read in place
    else:
        dy, ldy = _c(dy), N
    dx = torch.empty_like(x) if dx is None else dx
    if dx.is_contiguous():
        ldx = N
    elif dx.dim() == 2 and dx.shape == (M, N) and dx.stride(1) == 1:
        ldx = dx.stride(0)  # a column block of a wider gradient buffer (ops.PairFirstFn)
    else:
        raise ValueError(f"rmsnorm_bwd dx needs unit column stride, got {tuple(dx.stride())}")
    part = None
    if dw is not None:
        nb = nat.fns["sd_rmsnorm_bwd_blocks"](M, N)
        part = torch.empty(nb * N, dtype=torch.float32, device=x.device)
    nat.call("sd_rmsnorm_bwd_ldx", p(x), p(w), p(rstd), p(dy), ldy, p(dx), ldx, p(dw), p(part), M, N, int(act),
             int(accumulate_dx), int(accumulate_dw), stream())
    return dx


def colsum(x2d, out, accumulate=True):
    R, Nn = x2d.shape
    if x2d.stride(1) != 1:
        raise ValueError("colsum needs unit column stride")
    chunks = nat.fns["sd_colsum_chunks"](R)
    ws = torch.empty(chunks * Nn, dtype=torch.float32, device=x2d.device) if chunks > 1 else None
    nat.call("sd_colsum_ws", p(x2d), p(out), R, Nn, x2d.stride(0) if R > 1 else Nn, int(accumulate), p(ws),
             stream())
    return out


# ------------------------------------------------------------------------------------------------- latents
def seed_args(seed):
    """A sampling seed is an int, or a device int64 tensor (graph-replayable): -> (host part, device pointer)."""
    if isinstance(seed, torch.Tensor):
        return 0, seed.data_ptr()
    return int(seed) & 0xFFFFFFFFFFFFFFFF, 0


def onehot_sample(logits, K, unimix, seed, stream_id, step, group_offset, out=None, index=None, entropy=None):
    logits = _c(logits)
    groups = logits.numel() // K
    out = torch.empty_like(logits) if out is None else out
    sh, sp = seed_args(seed)
    nat.call("sd_onehot_sample_fwd", p(logits), p(out), p(index), p(entropy), groups, K, float(unimix),
             sh, int(stream_id), int(step), int(group_offset), sp, stream())
    return out


def onehot_entropy(logits, K, unimix):
    groups = logits.numel() // K
    ent = torch.empty(groups, dtype=torch.float32, device=logits.device)
    nat.call("sd_onehot_sample_fwd", p(_c(logits)), 0, 0, p(ent), groups, K, float(unimix), 0, 0, 0, 0, 0, stream())
    return ent


def onehot_sample_bwd(logits, dout, K, unimix, seed, stream_id, step, group_offset, dlogits=None, accumulate=False):
    groups = logits.numel() // K
    dlogits = torch.empty_like(logits) if dlogits is None else dlogits
    sh, sp = seed_args(seed)
    nat.call("sd_onehot_sample_bwd", p(_c(logits)), p(_c(dout)), p(dlogits), groups, K, float(unimix), sh,
             int(stream_id), int(step), int(group_offset), int(accumulate), sp, stream())
    return dlogits


def gru_fwd(gates, h, G, out=None):
    M, D = h.shape
    out = torch.empty_like(h) if out is None else out
    nat.call("sd_gru_fwd", p(_c(gates)), p(_c(h)), p(out), M, G, D // G, stream())
    return out


def gru_bwd(gates, h, dout, G, dgates=None, dh=None, accumulate_dh=False):
    M, D = h.shape
    dgates = torch.empty_like(gates) if dgates is None else dgates
    dh = torch.empty_like(h) if dh is None else dh
    nat.call("sd_gru_bwd", p(gates), p(h), p(_c(dout)), p(dgates), p(dh), M, G, D // G, int(accumulate_dh), stream())
    return dgates, dh


def action_norm(a, out=None):
    out = torch.empty_like(a) if out is None else out
    nat.call("sd_action_norm", p(_c(a)), p(out), a.numel(), stream())
    return out


def mask_rows(x, mask_u8, mask_stride=1, out=None):
    rows = mask_u8.numel() if mask_stride == 1 else x.shape[0]
    width = x.numel() // x.shape[0]
    out = torch.empty_like(x) if out is None else out
    nat.call("sd_mask_rows", p(_c(x)), p(mask_u8), int(mask_stride), p(out), x.shape[0], width, stream())
    return out


# ------------------------------------------------------------------------------------------------- heads
def twohot_mode(logits, bins, out=None):
    NB = logits.shape[-1]
    rows = logits.numel() // NB
    out = torch.empty(logits.shape[:-1] + (1,), dtype=torch.float32, device=logits.device) if out is None else out
    nat.call("sd_twohot_mode", p(_c(logits)), p(bins), p(out), rows, NB, stream())
    return out


def kl_rows(post, prior, S, K, free=None):
    """KL rows; with `free`, also the two free-nats clamped copies (dyn, rep) from the same launch."""
    rows = post.numel() // (S * K)
    out = torch.empty(rows if free is None else 3 * rows, dtype=torch.float32, device=post.device)
    kl = out[:rows]
    dyn, rep = (None, None) if free is None else (out[rows:2 * rows], out[2 * rows:])
    nat.call("sd_kl_fwd", p(_c(post)), p(_c(prior)), p(kl), p(dyn), p(rep), float(free or 0.0), rows, S, K, stream())
    return kl if free is None else (kl, dyn, rep)


def loss_terms(xs, coefs, scales, means, total):
    """sd_loss_terms_fwd: means (n,) (nullable) = coefs[i] * mean(xs[i]), total (1,) = sum scales[i] * means[i]"""
    L = nat.LossTerms()
    for i, x in enumerate(xs):
        t = L.t[i]
        t.x, t.n, t.coef, t.scale = p(_c(x)), x.numel(), float(coefs[i]), float(scales[i])
    L.n = len(xs)
    nat.call("sd_loss_terms_fwd", ctypes.addressof(L), p(means), p(total), stream())


def loss_terms_bwd(ns, coefs, scales, grads, g_total, g_means):
    """sd_loss_terms_bwd: grads[i] (ns[i] values, None = skipped) = (g_total scales[i] + g_means[i]) coefs[i] / ns[i]"""
    L = nat.LossTerms()
    for i, n in enumerate(ns):
        t = L.t[i]
        t.x, t.n, t.coef, t.scale, t.g = None, int(n), float(coefs[i]), float(scales[i]), p(grads[i])
    L.n = len(ns)
    nat.call("sd_loss_terms_bwd", ctypes.addressof(L), p(g_total), p(g_means), stream())


def device_mean(x):
    """mean of a contiguous f32 tensor as a 0-dim device tensor (one sd_loss_terms_fwd launch; no ATen reduce)"""
    out = torch.empty(1, dtype=torch.float32, device=x.device)
    loss_terms([_c(x)], [1.0], [1.0], None, out)
    return out[0]


def layout_copies(entries):
    """entries: (src, dst, batch, rows, cols, sb, sr, dcols, mode[, dld]) -> one sd_layout_copies_run launch"""
    L = nat.LayoutCopies()
    for i, ent in enumerate(entries):
        src, dst, batch, rows, cols, sb, sr, dcols, mode = ent[:9]
        e = L.e[i]
        e.src, e.dst, e.batch, e.rows, e.cols = p(src), p(dst), batch, rows, cols
        e.sb, e.sr, e.dcols, e.mode, e.dld = sb, sr, dcols, mode, (ent[9] if len(ent) > 9 else 0)
    L.n = len(entries)
    nat.call("sd_layout_copies_run", ctypes.addressof(L), stream())


def episode_flags(is_last, is_term):
    """bool (B, T[, 1]) -> f32 (B, T) last, term, cont = 1 - term (one launch)"""
    B, T = is_last.shape[:2]
    out = torch.empty(3, B, T, dtype=torch.float32, device=is_last.device)
    nat.call("sd_episode_flags", p(_c(is_last).view(torch.uint8)), p(_c(is_term).view(torch.uint8)), B * T,
             p(out[0]), p(out[1]), p(out[2]), stream())
    return out[0], out[1], out[2]


def lambda_return(reward, boot, disc, lamb, term=None, cont_logit=None, last=None, boot_row_stride=None,
                  boot_t_stride=1, cont_out=None, weight_out=None):
    """reward / cont_logit: (N, T) views of any strides (e.g. the transposed view of a time-major (T, N) tensor,
    read in place); boot: (row, t) strides given explicitly (default (T, 1)); term / last / outputs (N, T) row-major."""
    N, T = reward.shape
    ret = torch.empty(N, T - 1, dtype=torch.float32, device=reward.device)
    brs = T if boot_row_stride is None else boot_row_stride
    cs = cont_logit.stride() if cont_logit is not None else (T, 1)
    for t in (term, last, cont_out, weight_out):
        if t is not None:
            _c(t)
    nat.call("sd_lambda_return_strided", p(reward), reward.stride(0), reward.stride(1), p(term), p(cont_logit),
             cs[0], cs[1], p(last), p(boot), int(brs), int(boot_t_stride), p(ret), p(cont_out), p(weight_out), N, T,
             float(disc), float(lamb), stream())
    return ret


def return_ema(x, ema, offset_scale, quantiles=None, alpha=1e-2, q0=0.05, q1=0.95):
    x = _c(x)
    nat.call("sd_return_ema", p(x), x.numel(), p(ema), p(offset_scale), p(quantiles), float(alpha), float(q0),
             float(q1), stream())


def polyak(src, dst, mix):
    nat.call("sd_polyak", p(_c(src)), p(_c(dst)), src.numel(), float(mix), stream())


def u8_to_f32(img, shift=0.0, out=None):
    out = torch.empty(img.shape, dtype=torch.float32, device=img.device) if out is None else out
    nat.call("sd_u8_to_f32", p(_c(img)), p(out), img.numel(), float(shift), stream())
    return out


def u8_image_inputs(img, Cp, shift, need_f32=True):
    """uint8 (..., H, W, C) -> (img / 255 as f32 or None, encoder input img / 255 - shift padded to Cp channels), one
    launch"""
    C = img.shape[-1]
    pixels = img.numel() // C
    f = torch.empty(img.shape, dtype=torch.float32, device=img.device) if need_f32 else None
    enc = torch.empty(*img.shape[:-1], Cp, dtype=torch.float32, device=img.device)
    nat.call("sd_u8_image_inputs", p(_c(img)), p(f), p(enc), pixels, C, Cp, float(shift), stream())
    return f, enc


def pad_channels(x, Cp, shift=0.0):
    """NHWC (..., C) -> (..., Cp): x - shift, zero channels appended."""
    x = _c(x)
    C = x.shape[-1]
    out = torch.empty(*x.shape[:-1], Cp, dtype=torch.float32, device=x.device)
    nat.call("sd_pad_channels", p(x), p(out), x.numel() // C, C, Cp, float(shift), stream())
    return out


def symlog(x):
    y = torch.empty_like(x)
    nat.call("sd_symlog", p(_c(x)), p(y), x.numel(), stream())
    return y


def fill_gumbel(n, seed, stream_id, step, offset=0, device="cuda"):
    out = torch.empty(n, dtype=torch.float32, device=device)
    nat.call("sd_fill_gumbel", p(out), n, int(seed), int(stream_id), int(step), int(offset), stream())
    return out


def fill_normal(n, seed, stream_id, step, offset=0, device="cuda"):
    out = torch.empty(n, dtype=torch.float32, device=device)
    nat.call("sd_fill_normal", p(out), n, int(seed), int(stream_id), int(step), int(offset), stream())
    return out


# ------------------------------------------------------------------------------------------------- conv
def conv2d_fwd(x, w, b, ups=0, pad=None, out=None):
    """x (Nb, H, W, Ci) NHWC, w (Co, kh, kw, Ci) -> (Nb, H<<ups, W<<ups, Co)"""
    Nb, H, W, Ci = x.shape
    Co, kh, kw, _ = w.shape
    pad = (kh - 1) // 2 if pad is None else pad
    out = torch.empty(Nb, H << ups, W << ups, Co, dtype=torch.float32, device=x.device) if out is None else out
    nat.call("sd_conv2d_fwd", p(_c(x)), p(_c(w)), p(b), p(out), Nb, H, W, Ci, Co, kh, kw, pad, ups, stream())
    return out


def conv2d_dgrad(dout, w, pad=None, fast=True, direct=True):
    """Input gradient of a stride-1 conv: conv_same(dOut, flipped W). dout (Nb, H, W, Co), w (Co, kh, kw, Ci) ->
    (Nb, H, W, Ci). fast: split-bf16 MFMA kernels where their shape constraints hold — the direct kernel
    (sd_conv2d_dgrad_direct) first unless direct=False, then the implicit GEMM (sd_conv2d_dgrad_bf16x3)."""
    Co, kh, kw, Ci = w.shape
    pad = kh - 1 - (kh - 1) // 2 if pad is None else pad
    wf = _FLIP.get(w.data_ptr())
    if wf is None:
        wf = conv_flip_weight(w)
    if fast and FAST_GEMM:
        Nb, H, W, _ = dout.shape
        din = torch.empty(Nb, H, W, Ci, dtype=torch.float32, device=dout.device)
        if direct and DIRECT_DGRAD:  # the dOut patch staged once per workgroup (same products and order per k)
            ws = _SPLIT.get(w.data_ptr())
            if ws is None:
                ws = conv_split_weight(wf)
            if nat.call_shaped("sd_conv2d_dgrad_direct", p(_c(dout)), p(ws), p(din), Nb, H, W, Co, Ci, kh, kw, pad,
                               stream()):
                return din
        if nat.call_shaped("sd_conv2d_dgrad_bf16x3", p(_c(dout)), p(wf), p(din), Nb, H, W, Co, Ci, kh, kw, pad,
                           stream()):
            return din
    return conv2d_fwd(dout, wf, None, pad=pad)


def _wgrad_acc(acc):
    """(dw, db, ci_w) -> sd_wgrad_acc address (the launch adds [dW | db] into them), or None"""
    if acc is None:
        return None, None
    a = nat.WgradAcc()
    a.dw, a.db, a.ci_w = p(_c(acc[0])), p(_c(acc[1])), int(acc[2])
    return a, ctypes.addressof(a)


def conv2d_wgrad(x, dout, kh, kw, ups=0, pad=None, fast=True, acc=None):
    """returns (Co, kh*kw*Ci + 1) = [dW | db]. fast: split-bf16 direct kernel (sd_conv2d_wgrad_bf16x3) where eligible
    (Ci >= 16; the 4-channel first layer keeps the f32 direct kernel). acc = (dw, db, ci_w): the result is added into
    those parameter gradients by the launch's own reduction instead (returns None)."""
    Nb, H, W, Ci = x.shape
    Co = dout.shape[-1]
    pad = (kh - 1) // 2 if pad is None else pad
    J = kh * kw * Ci
    keep, ap = _wgrad_acc(acc)
    if fast and FAST_GEMM:
        ks = nat.fns["sd_conv2d_wgrad_bf16x3_slabs"](Nb, H, W, Ci, Co, kh, kw, ups)
        if ks > 0:
            out = torch.empty(Co, J + 1, dtype=torch.float32, device=x.device)
            ws = torch.empty(ks * Co * (J + 1), dtype=torch.float32, device=x.device) if ks > 1 else None
            if nat.call_shaped("sd_conv2d_wgrad_bf16x3", p(_c(x)), p(_c(dout)), p(out), p(ws),
                               ws.numel() if ws is not None else 0, Nb, H, W, Ci, Co, kh, kw, pad, ap, stream()):
                return None if acc is not None else out
    pixels = dout.numel() // Co
    ks = max(1, min(256, pixels // 4096))
    tiles = -(-Co // 64) * -(-(J + 1) // 64)
    ks = max(1, min(ks, max(1, 1024 // tiles)))
    out = torch.empty(Co, J + 1, dtype=torch.float32, device=x.device)
    ks = nat.fns["sd_conv2d_wgrad_slabs"](Nb, H, W, Ci, Co, kh, kw, ups, ks)
    ws = torch.empty(ks * Co * (J + 1), dtype=torch.float32, device=x.device) if ks > 1 else None
    nat.call("sd_conv2d_wgrad", p(_c(x)), p(_c(dout)), p(out), p(ws), ws.numel() if ws is not None else 0, ks,
             Nb, H, W, Ci, Co, kh, kw, pad, ups, ap, stream())
    del keep
    return None if acc is not None else out


def conv2d_wgrad_pool_slabs(x, Co, kh, kw):
    """> 0 when the pooled-gradient bwd-weight (sd_conv2d_wgrad_pool) handles this stage's shape."""
    Nb, H, W, Ci = x.shape
    return nat.fns["sd_conv2d_wgrad_pool_slabs"](Nb, H, W, Ci, Co, kh, kw)


# SDREAMER_WGRAD1_X3: the first encoder stage's bwd-weight (the pooled-gradient form) on the split-bf16 direct kernel
# (sd_conv2d_wgrad_pool_bf16x3) instead of the f32 one — the last f32 gradient contraction of the encoder, on the
# critical path (phase M2c). Default on (round 6: golden update + gradient tests green, LaProp moments as close to
# float64 as the f32 kernel's, profiles/r06f; update 10.91 -> 10.85 ms); 0 = the f32 kernel
WGRAD1_X3 = os.environ.get("SDREAMER_WGRAD1_X3", "1") == "1"


def conv2d_wgrad_pool(x, dpool, amax, kh, kw, pad=None, acc=None):
    """[dW | db] (Co, kh*kw*Ci + 1) of a pooled stage from the max-pool backward's pooled-resolution gradient and the
    forward's argmax (the f32 direct kernel expands them while staging; the same products as conv2d_wgrad on the
    expanded gradient, summed in 512-pixel row blocks instead of 128: reordered f32 sums, ~2e-5 relative). With
    WGRAD1_X3 the split-bf16 direct kernel where its plan takes the shape (~1e-5 of sum |a b| per element)."""
    Nb, H, W, Ci = x.shape
    Co = dpool.shape[-1]
    pad = (kh - 1) // 2 if pad is None else pad
    J = kh * kw * Ci
    if WGRAD1_X3 and FAST_GEMM:
        ks = nat.fns["sd_conv2d_wgrad_pool_bf16x3_slabs"](Nb, H, W, Ci, Co, kh, kw)
        if ks > 0:
            out = torch.empty(Co, J + 1, dtype=torch.float32, device=x.device)
            ws = torch.empty(ks * Co * (J + 1), dtype=torch.float32, device=x.device)
            keep, ap = _wgrad_acc(acc)
            nat.call("sd_conv2d_wgrad_pool_bf16x3", p(_c(x)), p(_c(dpool)), p(_c(amax)), p(out), p(ws), ws.numel(),
                     Nb, H, W, Ci, Co, kh, kw, pad, ap, stream())
            del keep
            return None if acc is not None else out
    ks = conv2d_wgrad_pool_slabs(x, Co, kh, kw)
    if ks <= 0:
        raise nat.NativeError("sd_conv2d_wgrad_pool: shape outside the direct kernel")
    out = torch.empty(Co, J + 1, dtype=torch.float32, device=x.device)
    ws = torch.empty(ks * Co * (J + 1), dtype=torch.float32, device=x.device)
    keep, ap = _wgrad_acc(acc)
    nat.call("sd_conv2d_wgrad_pool", p(_c(x)), p(_c(dpool)), p(_c(amax)), p(out), p(ws), ws.numel(), Nb, H, W, Ci, Co,
             kh, kw, pad, ap, stream())
    del keep
    return None if acc is not None else out


_FLIP = {}  # weight data_ptr -> flipped weight, built ahead of the backward (set_flip_cache)
_SPLIT = {}  # weight data_ptr -> split-bf16 image of the flipped weight (sd_conv_split_weight), same lifetime
# SDREAMER_CONV6: the encoder stages' forward on the fp32-accurate three-way split-bf16 direct kernel
# (sd_conv2d_fwd_pool6, the weight through an LDS ring) instead of the exact f32 kernels. Default "1": every
# instantiated stage — 32 -> 48 channels at 32 x 32 (0.67 -> 0.40 ms) and 48 -> 64 at 16 x 16 (0.38 -> 0.19 ms,
# profiles/r06s3b); "s2" the first of them only, "0" none. Round 6 measured its parity against exact arithmetic
# (tools/precision_study.py over the golden cases' LaProp moments, profiles/r06f, r06s3b): it sits as close to the
# float64 answer as the f32 kernels do in every golden case, and closer where the reference's own f32 is far from it
# (walker_r2_nowarm's first conv layer: 0.02 of the bound from float64, the reference 5.1; the golden update test
# accepts the reference's answer or exact arithmetic per tensor there).
CONV6 = os.environ.get("SDREAMER_CONV6", "1")
CONV6 = CONV6 if CONV6 in ("1", "s2") else ""
# SDREAMER_DIRECT_DGRAD=0: the encoder's bwd-data on the implicit-GEMM split-bf16 kernel (A/B knob)
DIRECT_DGRAD = os.environ.get("SDREAMER_DIRECT_DGRAD", "1") != "0"


def set_flip_cache(weights):
    """Flip conv weights for conv2d_dgrad ahead of time (Dreamer builds them on the main stream while it waits for
    the imagined returns, off the encoder backward's chain); valid until clear_flip_cache (the optimizer step changes
    the weights). Returns the flipped tensors (the caller keeps them alive)."""
    _FLIP.clear()
    _SPLIT.clear()
    for w in weights:
        _FLIP[w.data_ptr()] = conv_flip_weight(w)
        if FAST_GEMM and DIRECT_DGRAD:
            _SPLIT[w.data_ptr()] = conv_split_weight(_FLIP[w.data_ptr()])
    return list(_FLIP.values()) + list(_SPLIT.values())


def clear_flip_cache():
    _FLIP.clear()
    _SPLIT.clear()


def conv_split_weight(wf):
    """[plane][Ci][KP] bf16 (hi, lo) image of a flipped weight wf (Ci, kh, kw, Co), KP = kh*kw*Co rounded up to 32
    (sd_conv_split_weight), the B operand of sd_conv2d_dgrad_direct; held as int16 storage."""
    rows, K = wf.shape[0], wf[0].numel()
    KP = -(-K // 32) * 32
    ws = torch.empty(2 * rows * KP, dtype=torch.int16, device=wf.device)
    nat.call("sd_conv_split_weight", p(_c(wf)), p(ws), rows, K, stream())
    return ws


def conv_flip_weight(w):
    Co, kh, kw, Ci = w.shape
    wf = torch.empty(Ci, kh, kw, Co, dtype=torch.float32, device=w.device)
    nat.call("sd_conv_flip_weight", p(_c(w)), p(wf), Co, kh, kw, Ci, stream())
    return wf


def random_translate(img, pad, seed, row_offset=0, same_across_time=True, bilinear=True):
    """Dreamer.random_translate (dreamer.py:845-880) on preprocessed (B, T, H, W, C) f32 images (NHWC, as the
    reference permutes back): replicate pad + Philox integer shift per slice row (or per image), sampled like the
    reference's grid_sample (bilinear: its f32 grid arithmetic, bit-exact with torch's CPU kernel; else nearest)."""
    B, T, H, W, C = img.shape
    out = torch.empty_like(img)
    sh, sp = seed_args(seed)
    nat.call("sd_random_translate", p(_c(img)), p(out), B, T, H, W, C, int(pad), sh, sp, int(row_offset),
             int(bool(same_across_time)), int(bool(bilinear)), stream())
    return out


def sumpool2(du):
    Nb, H2, W2, C = du.shape
    din = torch.empty(Nb, H2 // 2, W2 // 2, C, dtype=torch.float32, device=du.device)
    nat.call("sd_sumpool2", p(_c(du)), p(din), Nb, H2 // 2, W2 // 2, C, stream())
    return din


def pool_rms_fwd(x, w, nchw_flat=False):
    Nb, H, W, C = x.shape
    pooled = torch.empty(Nb, H // 2, W // 2, C, dtype=torch.float32, device=x.device)
    amax = torch.empty(Nb, H // 2, W // 2, C, dtype=torch.uint8, device=x.device)
    y = torch.empty_like(pooled)
    rstd = torch.empty(Nb, H // 2, W // 2, dtype=torch.float32, device=x.device)
    nat.call("sd_pool_rms_fwd", p(_c(x)), p(w), p(pooled), p(amax), p(y), p(rstd), Nb, H, W, C, EPS, int(nchw_flat),
             stream())
    return y, pooled, amax, rstd


def ops_fused_pool():
    from . import ops
    return ops.FUSED_POOL


def conv2d_fwd_pool(x, w, b, nw, nchw_flat=False):
    """Fused ConvEncoder stage forward (sd_conv2d_fwd_pool): x (Nb, H, W, Ci) NHWC, w (Co, kh, kw, Ci) ->
    (y, pooled, amax, rstd) as pool_rms_fwd(conv2d_fwd(x, w, b), nw) returns them, or None when the shape is outside
    the fused kernel."""
    Nb, H, W, Ci = x.shape
    Co, kh, kw, _ = w.shape
    pooled = torch.empty(Nb, H // 2, W // 2, Co, dtype=torch.float32, device=x.device)
    amax = torch.empty(Nb, H // 2, W // 2, Co, dtype=torch.uint8, device=x.device)
    y = torch.empty_like(pooled)
    rstd = torch.empty(Nb, H // 2, W // 2, dtype=torch.float32, device=x.device)
    if CONV6 and (CONV6 == "1" or (Ci, Co) == (32, 48)):  # fp32-accurate three-way split-bf16 direct kernel
        K = kh * kw * Ci
        ws = torch.empty(3 * Co * (-(-K // 32) * 32), dtype=torch.int16, device=x.device)
        nat.call("sd_conv_split3_weight", p(_c(w)), p(ws), Co, K, stream())
        if nat.call_shaped("sd_conv2d_fwd_pool6", p(_c(x)), p(ws), p(b), p(nw), p(pooled), p(amax), p(y), p(rstd),
                           Nb, H, W, Ci, Co, kh, kw, (kh - 1) // 2, EPS, int(nchw_flat), stream()):
            return y, pooled, amax, rstd
    ok = nat.call_shaped("sd_conv2d_fwd_pool", p(_c(x)), p(_c(w)), p(b), p(nw), p(pooled), p(amax), p(y), p(rstd),
                         Nb, H, W, Ci, Co, kh, kw, (kh - 1) // 2, EPS, int(nchw_flat), stream())
    return (y, pooled, amax, rstd) if ok else None


def pool_rms_bwd_compact(pooled, amax, w, rstd, dy, dw, nchw_flat=False):
    """pool_rms_bwd writing the pooled-resolution gradient (Nb, H/2, W/2, C) instead of the scattered conv gradient."""
    Nb, Ho, Wo, C = pooled.shape
    H, W = 2 * Ho, 2 * Wo
    dp = torch.empty_like(pooled)
    nb = nat.fns["sd_pool_rms_bwd_blocks"](Nb, H, W)
    part = torch.empty((nb + nat.fns["sd_colsum_chunks"](nb)) * C, dtype=torch.float32, device=pooled.device)
    nat.call("sd_pool_rms_bwd_compact", p(pooled), p(amax), p(w), p(rstd), p(_c(dy)), p(dp), p(dw), p(part), Nb, H, W,
             C, int(nchw_flat), 1, stream())
    return dp


def pool_rms_bwd(pooled, amax, w, rstd, dy, H, W, dw, nchw_flat=False):
    Nb, Ho, Wo, C = pooled.shape
    dx = torch.empty(Nb, H, W, C, dtype=torch.float32, device=pooled.device)
    nb = nat.fns["sd_pool_rms_bwd_blocks"](Nb, H, W)
    part = torch.empty((nb + nat.fns["sd_colsum_chunks"](nb)) * C, dtype=torch.float32, device=pooled.device)
    nat.call("sd_pool_rms_bwd", p(pooled), p(amax), p(w), p(rstd), p(_c(dy)), p(dx), p(dw), p(part), Nb, H, W, C,
             int(nchw_flat), 1, stream())
    return dx


# ------------------------------------------------------------------------------------------------- timeline marks
class Marks:
    """Device timestamps (sd_mark) at tagged points of the update, on whatever stream is current — captured into the
    HIP graph like any launch, so replayed updates report the real two-stream timeline. Profiling aid only."""

    def __init__(self, device, slots=256):
        self.buf = torch.zeros(slots, dtype=torch.int64, device=device)
        self.tags = []
        self.khz = nat.fns["sd_wall_clock_khz"](torch.device(device).index or 0)

    def reset(self):
        self.tags = []

    def __call__(self, tag):
        if len(self.tags) >= self.buf.numel():
            return
        nat.call("sd_mark", p(self.buf), len(self.tags), stream())
        self.tags.append(tag)

    def report(self):
        """[(tag, microseconds since the first mark)] of the last completed update"""
        v = self.buf[:len(self.tags)].cpu().tolist()
        return [(t, (x - v[0]) * 1e3 / self.khz) for t, x in zip(self.tags, v)]


# ------------------------------------------------------------------------------------------------- launch probe
class LaunchProbe:
    """Times every launch of one C-ABI entry point (filtered by its arguments) with HIP events recorded on the
    stream the kernel is launched on (torch's current stream). Used by bench.py for the roofline fraction."""

    def __init__(self, name, pred, work_fn, bound="mfma", unit="TFLOP/s", peak=157.3, label=""):
        self.name, self.pred, self.work_fn = name, pred, work_fn
        self.bound, self.unit, self.peak, self.label = bound, unit, peak, label
        self.records = []
        self._start = None
        nat.PROBES.append(self)

    def match(self, name, args):
        return name == self.name and self.pred(args)

    def end(self, args):
        e = torch.cuda.Event(enable_timing=True)
        if torch.cuda.is_current_stream_capturing():
            self.captured_args = args  # inside a HIP-graph capture: remember the launch, time it by replay()
            self._start = None
            return
        e.record()
        self.records.append((self._start, e, self.work_fn(args)))
        self.captured_args = args

    def begin(self):
        if torch.cuda.is_current_stream_capturing():
            return
        self._start = torch.cuda.Event(enable_timing=True)
        self._start.record()

    def replay(self, n=20):
        """Re-issue the last recorded launch (same buffers, same shapes) n times, each bracketed by HIP events on
        the current stream (graph-replayed steps are invisible to Python-side hooks)."""
        args = getattr(self, "captured_args", None)
        if args is None:
            return
        args = tuple(args[:-1]) + (stream(),)  # launch on the stream the events are recorded on
        self.records = []
        for _ in range(n):
            s = torch.cuda.Event(enable_timing=True)
            e = torch.cuda.Event(enable_timing=True)
            s.record()
            nat.check(nat.fns[self.name](*args), self.name)
            e.record()
            self.records.append((s, e, self.work_fn(args)))
        torch.cuda.synchronize()

    def stop(self):
        if self in nat.PROBES:
            nat.PROBES.remove(self)
        torch.cuda.synchronize()

    def report(self):
        if not self.records:
            return None
        ms = [s.elapsed_time(e) for s, e, _ in self.records]
        work = [w for _, _, w in self.records]
        avg_ms = sum(ms) / len(ms)
        per_launch = sum(work) / len(work)
        achieved = per_launch / (avg_ms * 1e-3) / (1e12 if self.unit == "TFLOP/s" else 1e9)
        return {"bound": self.bound, "achieved": achieved, "peak": self.peak, "unit": self.unit,
                "frac": achieved / self.peak, "traffic": None, "kernel": self.label, "launches": len(ms),
                "avg_us": avg_ms * 1e3, "work_per_launch": per_launch}


# ------------------------------------------------------------------------------------------------- metrics
STAT_MEAN, STAT_STD, STAT_MIN, STAT_MAX = 0, 1, 2, 3
_STAT_CHUNK = nat._define(nat.HEADER, "SD_STAT_CHUNK")


class Stat:
    """A metric resolved later, with every other metric of the update, by ONE sd_multi_stats launch: a sum of
    scale * stat(tensor) terms (stat: mean, unbiased std, min, max of the whole tensor; a scalar is its own mean)."""

    __slots__ = ("terms", "affine")

    def __init__(self, t, kind=STAT_MEAN, scale=1.0, sub=None, div=None):
        self.terms = [(t, int(kind), float(scale))]
        self.affine = (sub, div)  # device scalars: (stat - sub) / div, applied to a single-term Stat

    def __add__(self, other):
        r = Stat.__new__(Stat)
        if self.affine != (None, None) or (isinstance(other, Stat) and other.affine != (None, None)):
            raise ValueError("an affine Stat is a metric of its own")
        r.terms = self.terms + (other.terms if isinstance(other, Stat) else Stat(other).terms)
        r.affine = (None, None)
        return r

    __radd__ = __add__

    def __mul__(self, k):
        r = Stat.__new__(Stat)
        r.terms = [(t, kind, sc * float(k)) for t, kind, sc in self.terms]
        r.affine = self.affine
        return r

    __rmul__ = __mul__

    def record_stream(self, s):
        for t, _, _ in self.terms:
            t.record_stream(s)
        for t in self.affine:
            if t is not None:
                t.record_stream(s)


def tensorstats(t, prefix):
    """tools.tensorstats (tools.py:275-281) as lazy metrics"""
    t = t.detach()
    return {f"{prefix}_mean": Stat(t, STAT_MEAN), f"{prefix}_std": Stat(t, STAT_STD),
            f"{prefix}_min": Stat(t, STAT_MIN), f"{prefix}_max": Stat(t, STAT_MAX)}


def metric_vector(values):
    """(len(values),) float32 device tensor: values are Stat or tensors (a tensor = its mean); one sd_multi_stats call
    (two launches) per SD_MAX_STATS terms (normally one)."""
    reqs, empty = [], []
    for i, v in enumerate(values):
        aff = v.affine if isinstance(v, Stat) else (None, None)
        for t, kind, sc in (v.terms if isinstance(v, Stat) else [(v, STAT_MEAN, 1.0)]):
            t = t.detach()
            if t.numel() == 0:  # torch semantics: mean / std / min / max of nothing is NaN (sd_multi_stats needs n > 0)
                empty.append(i)
                continue
            if t.dtype != torch.float32:
                t = t.float()
            reqs.append((_c(t), kind, sc, i, aff))
    out = torch.empty(len(values), dtype=torch.float32, device=reqs[0][0].device if reqs else "cuda")
    if not reqs:
        return out.fill_(float("nan"))
    cap = len(nat.Stats().r)
    chunk = _STAT_CHUNK
    for lo in range(0, len(reqs), cap):
        st = nat.Stats()
        part = reqs[lo:lo + cap]
        c0 = 0
        for j, (t, kind, sc, i, aff) in enumerate(part):
            r = st.r[j]
            r.x, r.n, r.kind, r.out, r.scale, r.chunk0 = p(t), t.numel(), kind, i, sc, c0
            r.sub, r.div = p(aff[0]), p(aff[1])
            c0 += (t.numel() + chunk - 1) // chunk
        st.nreq = len(part)
        ws = torch.empty(5 * c0, dtype=torch.float32, device=out.device)
        dst = out if lo == 0 else torch.empty_like(out)
        nat.call("sd_multi_stats", ctypes.addressof(st), p(ws), p(dst), len(values), stream())
        if lo:  # a second table's slots add to the first's
            out.add_(dst)
    for i in sorted(set(empty)):  # no host-to-device index copy: capture-safe (the S2 phase graph builds metrics)
        out[i:i + 1].fill_(float("nan"))
    return out


def resolve_metrics(mets):
    """dict with Stat values -> dict of 0-dim device tensors (one launch for all of them)"""
    keys = [k for k, v in mets.items() if isinstance(v, (Stat, torch.Tensor))]
    vec = metric_vector([mets[k] for k in keys])
    out = dict(mets)
    for i, k in enumerate(keys):
        out[k] = vec[i]
    return out
