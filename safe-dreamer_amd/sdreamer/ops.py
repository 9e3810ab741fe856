"""Autograd wrappers: each differentiable piece of the update owns a HIP forward AND a HIP backward.

Parameter gradients are accumulated straight into `param.grad` (normally a view into the flat gradient arena,
see sdreamer/optim.py) by the backward kernels (GEMM beta=1 / accumulate flags) instead of being returned to
autograd, so weight gradients never take an extra allocation + add pass. Input gradients are returned normally.
"""
from __future__ import annotations

import os

import torch

from . import kernels as k


# ConvEncoder stages run conv + pool + norm as one launch where the shape allows (SDREAMER_FUSED_POOL=0: two launches)
FUSED_POOL = os.environ.get("SDREAMER_FUSED_POOL", "1") != "0"


def grad_buf(param):
    if param.grad is None:
        param.grad = torch.zeros_like(param)
    return param.grad


def _flat(x):
    return x.reshape(-1, x.shape[-1])


# ------------------------------------------------------------------------------------------------- dense layers
_DEFER = None  # a list while defer_wgrads is active


class defer_wgrads:
    """Within this context LinearFn's backward computes the input gradient immediately and queues its weight / bias
    gradient contractions in `bucket`; flush_wgrads runs them later, possibly on another stream (the replay-value
    loss's value-head weight gradients run on the side stream, off the path to the posterior backward)."""

    def __init__(self, bucket):
        self.bucket = bucket

    def __enter__(self):
        global _DEFER
        self.prev, _DEFER = _DEFER, self.bucket
        return self.bucket

    def __exit__(self, *exc):
        global _DEFER
        _DEFER = self.prev


def flush_wgrads(bucket):
    """Run the queued weight-gradient work on the current stream (inputs marked as used by it)."""
    st = torch.cuda.current_stream()
    eager = not torch.cuda.is_current_stream_capturing()  # captured phases keep their tensors in the graph pools
    for fn, tensors in bucket:
        if eager:
            for t in tensors:
                t.record_stream(st)
        fn()
    bucket.clear()


class DxSink:
    """One input-gradient buffer shared by several linear layers that read the same tensor x (the world-model heads
    and the replay value head on the posterior feat, dreamer.py:571-660): each layer's backward adds its x gradient
    into `buf` inside its own GEMM (beta = 1 after the first writer) and returns no gradient to autograd, so the
    pairwise autograd adds, the slice-backward copies of the concatenated feat and the leaf-gradient copies are never
    launched. Mark an input with `sink(x, s)`; `written` tells whether any layer's gradient arrived."""

    def __init__(self, like):
        self.buf = torch.empty(like.shape, dtype=torch.float32, device=like.device)
        self.written = False


def sink(x, s):
    """x with its linear layers' input gradients routed into DxSink s (the attribute does not survive a view)"""
    x._dx_sink = s
    return x


class LinearFn(torch.autograd.Function):
    """nn.Linear (y = x W^T + b). Gradients on the split-bf16 GEMM (k.gemm fast=True, ~1e-5 relative); the forward
    too when `fast` (imagined-trajectory heads: no sampled index depends on them). An input marked with a DxSink gets
    its gradient accumulated there instead of returned."""

    @staticmethod
    def forward(ctx, x, w, b, fast=False):
        x2 = _flat(x).contiguous()
        y = k.mm(x2, w.t(), bias=b, fast=fast)
        ctx.save_for_backward(x2, w, b)
        ctx.in_shape = x.shape
        ctx.dx_sink = getattr(x, "_dx_sink", None)
        return y.view(*x.shape[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x2, w, b = ctx.saved_tensors
        dy2 = _flat(dy).contiguous()
        dx = None
        sk = ctx.dx_sink
        if sk is not None:
            k.mm(dy2, w, out=sk.buf.view(-1, w.shape[1]), beta=1.0 if sk.written else 0.0, fast=True)
            sk.written = True
        elif ctx.needs_input_grad[0]:
            dx = k.mm(dy2, w, fast=True).view(ctx.in_shape)

        def wgrad():
            if w.requires_grad:  # dW (+ db in the same launch)
                k.wgrad(dy2, x2, grad_buf(w), grad_buf(b) if (b is not None and b.requires_grad) else None)
            elif b is not None and b.requires_grad:
                k.colsum(dy2, grad_buf(b), accumulate=True)

        if _DEFER is not None:
            _DEFER.append((wgrad, (dy2, x2)))
        else:
            wgrad()
        return dx, None, None, None


class LinearPreFn(torch.autograd.Function):
    """A linear layer whose forward output h = x W^T + b was already computed elsewhere (the imagination's fp32 actor
    layer 0, the imagined heads' batched first layers): forward returns h0 as the layer's output, backward accumulates
    the weight / bias gradients exactly as LinearFn does (split-bf16 dW = dh^T x, column sums for db). x is a detached
    input (imagined features): no input gradient."""

    @staticmethod
    def forward(ctx, h0, x, w, b):
        ctx.save_for_backward(_flat(x).contiguous(), w, b)
        return h0.view_as(h0)

    @staticmethod
    def backward(ctx, dy):
        x2, w, b = ctx.saved_tensors
        dy2 = _flat(dy).contiguous()

        def wgrad():
            if w.requires_grad:  # dW (+ db in the same launch)
                k.wgrad(dy2, x2, grad_buf(w), grad_buf(b) if (b is not None and b.requires_grad) else None)
            elif b is not None and b.requires_grad:
                k.colsum(dy2, grad_buf(b), accumulate=True)

        if _DEFER is not None:
            _DEFER.append((wgrad, (dy2, x2)))
        else:
            wgrad()
        return None, None, None, None


class PairFirstFn(torch.autograd.Function):
    """The first layer (Linear -> RMSNorm -> SiLU) of two MLPs on the same detached input x whose linear outputs
    h0a, h0b were computed elsewhere: the imagined actor's (the imagination's fp32 layer 0) and the value head's (the
    imagined heads' batched first layer), dreamer.py:607,613. Forward = the two norms (as RmsSiluFn). Backward: both
    norms' input gradients into the two column blocks of one (R, Ua + Ub) buffer, then ONE split-bf16 weight-gradient
    GEMM over it (sd_gemm_bf16x3_wgrad2) — x (H*N x feat, 157 MB at the bench config) is read once instead of once per
    head, and its K chunks are twice as long. The two weight gradients must lie back to back (Dreamer._arena_order);
    otherwise two GEMMs over the buffer's column blocks."""

    @staticmethod
    def forward(ctx, h0a, h0b, x, wa, ba, na, wb, bb, nb):
        h0a, h0b = h0a.contiguous(), h0b.contiguous()
        ya, ra = k.rmsnorm_fwd(h0a, na, act=1)
        yb, rb = k.rmsnorm_fwd(h0b, nb, act=1)
        ctx.save_for_backward(h0a, h0b, ra, rb, _flat(x).contiguous(), wa, ba, na, wb, bb, nb)
        return ya, yb

    @staticmethod
    def backward(ctx, dya, dyb):
        h0a, h0b, ra, rb, x2, wa, ba, na, wb, bb, nb = ctx.saved_tensors
        R, Ua = h0a.shape
        Ub = h0b.shape[1]
        buf = torch.empty(R, Ua + Ub, dtype=torch.float32, device=h0a.device)
        for h0, nw, r, dy, cols in ((h0a, na, ra, dya, slice(0, Ua)), (h0b, nb, rb, dyb, slice(Ua, Ua + Ub))):
            if dy is None:
                buf[:, cols].zero_()
            else:
                k.rmsnorm_bwd(h0, nw, r, dy, act=1, dx=buf[:, cols], dw=grad_buf(nw) if nw.requires_grad else None)

        def wgrad():
            ga, gb = grad_buf(wa), grad_buf(wb)
            if not (gb.data_ptr() == ga.data_ptr() + ga.numel() * ga.element_size() and ga.is_contiguous() and
                    gb.is_contiguous() and k.wgrad2(buf, x2, ga.as_strided((Ua + Ub, ga.shape[1]), (ga.shape[1], 1)),
                                                    grad_buf(ba), grad_buf(bb), Ua) is not False):
                k.wgrad(buf[:, :Ua], x2, ga, grad_buf(ba))
                k.wgrad(buf[:, Ua:], x2, gb, grad_buf(bb))

        if _DEFER is not None:
            _DEFER.append((wgrad, (buf, x2)))
        else:
            wgrad()
        return (None,) * 9


class RmsSiluFn(torch.autograd.Function):
    """nn.RMSNorm(eps=1e-4) followed by SiLU (act=1) or nothing (act=0)."""

    @staticmethod
    def forward(ctx, x, w, act):
        x = x.contiguous()
        y, rstd = k.rmsnorm_fwd(x, w, act=act)
        ctx.save_for_backward(x, w, rstd)
        ctx.act = act
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, rstd = ctx.saved_tensors
        dw = grad_buf(w) if w.requires_grad else None
        dx = k.rmsnorm_bwd(x, w, rstd, dy.contiguous(), act=ctx.act, dw=dw)
        return dx, None, None


class BlockLinearFn(torch.autograd.Function):
    """BlockLinear (networks.py:24-56) with the weight kept packed as (G, O/G, I/G)."""

    @staticmethod
    def forward(ctx, x, wp, b):
        G, Og, Ig = wp.shape
        x2 = _flat(x).contiguous()
        M = x2.shape[0]
        y = torch.empty(M, G * Og, dtype=torch.float32, device=x.device)
        k.gemm(x2.view(M, G, Ig).permute(1, 0, 2), wp.transpose(1, 2), y.view(M, G, Og).permute(1, 0, 2),
               bias=b.view(G, Og))
        ctx.save_for_backward(x2, wp, b)
        ctx.in_shape = x.shape
        return y.view(*x.shape[:-1], G * Og)

    @staticmethod
    def backward(ctx, dy):
        x2, wp, b = ctx.saved_tensors
        G, Og, Ig = wp.shape
        M = x2.shape[0]
        dy2 = _flat(dy).contiguous()
        dyv = dy2.view(M, G, Og).permute(1, 0, 2)
        dx = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty(M, G * Ig, dtype=torch.float32, device=dy.device)
            k.gemm(dyv, wp, dx.view(M, G, Ig).permute(1, 0, 2), fast=True)
            dx = dx.view(ctx.in_shape)
        if wp.requires_grad:
            k.gemm(dyv.transpose(1, 2), x2.view(M, G, Ig).permute(1, 0, 2), grad_buf(wp), beta=1.0, fast=True)
        if b.requires_grad:
            k.colsum(dy2, grad_buf(b), accumulate=True)
        return dx, None, None


def linear(x, w, b=None, fast=False):
    return LinearFn.apply(x, w, b, fast)


def linear_pre(h0, x, w, b=None):
    return LinearPreFn.apply(h0, x, w, b)


def rms_silu(x, w, act=1):
    return RmsSiluFn.apply(x, w, act)


def block_linear(x, wp, b):
    return BlockLinearFn.apply(x, wp, b)


# ------------------------------------------------------------------------------------------------- conv
# SDREAMER_POOL_COMPACT=0: first-stage backward through the full-resolution conv gradient (benchmark / test knob)
POOL_COMPACT = os.environ.get("SDREAMER_POOL_COMPACT", "1") != "0"


class CatIntoFn(torch.autograd.Function):
    """torch.cat([a, b], -1) written into a caller-owned buffer (holder[0]) and returned with autograd: RSSM.get_feat
    (rssm.py:211-217) straight into the imagination's start slot, so the start state is never copied again."""

    @staticmethod
    def forward(ctx, a, b, holder):
        out = holder[0]
        na, nb, F = a.shape[-1], b.shape[-1], out.shape[-1]
        rows = a.numel() // na
        if out.stride(-1) != 1 or out.numel() != rows * F or na + nb != F or not (a.is_contiguous() and b.is_contiguous()):
            torch.cat([a, b], -1, out=out)
        else:  # both halves in one sd_layout_copies_run launch (row stride F into the slot)
            base = out.reshape(rows, F)
            k.layout_copies([(a, base, 1, rows, na, 0, na, na, 1, F), (b, base[:, na:], 1, rows, nb, 0, nb, nb, 1, F)])
        ctx.split = na
        ctx.set_materialize_grads(False)  # consumers that route their gradient into a DxSink send none here
        return out

    @staticmethod
    def backward(ctx, g):
        if g is None:
            return None, None, None
        return g[..., :ctx.split], g[..., ctx.split:], None


def _pad_last(w, n):
    """w (..., c) -> (..., n) zero-padded, one sd_layout_copies_run launch"""
    wc = w.contiguous()
    out = torch.empty(*w.shape[:-1], n, dtype=w.dtype, device=w.device)
    rows = wc.numel() // w.shape[-1]
    k.layout_copies([(wc, out, 1, rows, w.shape[-1], 0, w.shape[-1], n, 1)])
    return out


class ConvPoolNormFn(torch.autograd.Function):
    """One ConvEncoder stage: Conv2dSamePad -> MaxPool2d(2) -> RMSNorm2D -> SiLU (networks.py:201-216), NHWC.
    Forward on the exact f32 MFMA kernels (the posterior samples depend on it); both backward contractions on the
    split-bf16 kernels (k.conv2d_wgrad / k.conv2d_dgrad, ~1e-5 relative)."""

    @staticmethod
    def forward(ctx, x, w, b, nw, nchw_flat):
        # x may carry zero-padded channels (first layer: 3 -> 4); the weight is padded to match
        wk = w if x.shape[-1] == w.shape[-1] else _pad_last(w, x.shape[-1])
        fused = k.conv2d_fwd_pool(x.contiguous(), wk, b, nw, nchw_flat=nchw_flat) if FUSED_POOL else None
        if fused is None:
            conv = k.conv2d_fwd(x.contiguous(), wk, b)
            fused = k.pool_rms_fwd(conv, nw, nchw_flat=nchw_flat)
            del conv
        y, pooled, amax, rstd = fused
        ctx.save_for_backward(x, w, b, nw, pooled, amax, rstd)
        ctx.nchw_flat = nchw_flat
        if nchw_flat:
            return y.view(y.shape[0], -1)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, b, nw, pooled, amax, rstd = ctx.saved_tensors
        Nb, H, W, _ = x.shape
        Co, kh, kw, Ci = w.shape
        acc = (grad_buf(w), grad_buf(b), Ci)  # the bwd-weight launches add into the gradients themselves
        if not ctx.needs_input_grad[0] and POOL_COMPACT and k.conv2d_wgrad_pool_slabs(x, Co, kh, kw) > 0:
            # first stage (no input gradient): the bwd-weight kernel expands the pooled gradient + argmax itself, so
            # the full-resolution conv gradient (3/4 zeros) is never written or read
            dpool = k.pool_rms_bwd_compact(pooled, amax, nw, rstd, dy.contiguous(), grad_buf(nw), nchw_flat=ctx.nchw_flat)
            k.conv2d_wgrad_pool(x, dpool, amax, kh, kw, acc=acc)
            dconv = None
        else:
            dconv = k.pool_rms_bwd(pooled, amax, nw, rstd, dy.contiguous(), H, W, grad_buf(nw), nchw_flat=ctx.nchw_flat)
        Cx = x.shape[-1]

        def wgrad():
            k.conv2d_wgrad(x, dconv, kh, kw, acc=acc)

        if dconv is None:
            pass
        elif _DEFER is not None:  # queued: only the data gradient continues the backward chain
            _DEFER.append((wgrad, (x, dconv)))
        else:
            wgrad()
        dx = None
        if ctx.needs_input_grad[0]:
            if Cx != Ci:
                raise NotImplementedError("input gradient through a channel-padded conv")
            dx = k.conv2d_dgrad(dconv, w)
        return dx, None, None, None, None


class UpConvFn(torch.autograd.Function):
    """nn.Upsample(2, nearest) -> Conv2dSamePad (ConvDecoder, networks.py:259-265), NHWC, no materialised upsample."""

    @staticmethod
    def forward(ctx, x, w, b):
        y = k.conv2d_fwd(x.contiguous(), w, b, ups=1)
        ctx.save_for_backward(x, w, b)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, b = ctx.saved_tensors
        Co, kh, kw, Ci = w.shape
        dy = dy.contiguous()
        k.conv2d_wgrad(x, dy, kh, kw, ups=1, acc=(grad_buf(w), grad_buf(b), Ci))
        dx = None
        if ctx.needs_input_grad[0]:
            du = k.conv2d_dgrad(dy, w)
            dx = k.sumpool2(du)
        return dx, None, None


# ------------------------------------------------------------------------------------------------- distributions
class KLFn(torch.autograd.Function):
    """RSSM.kl_loss (rssm.py:222-230): returns (dyn_row, rep_row) = clip(sum_S KL, min=free) for every row."""

    @staticmethod
    def forward(ctx, post, prior, free, S, K):
        post, prior = post.contiguous(), prior.contiguous()
        kl, dyn, rep = k.kl_rows(post, prior, S, K, free=free)  # the clamped copies come from the same launch
        ctx.set_materialize_grads(False)
        ctx.save_for_backward(post, prior, kl)
        ctx.free, ctx.S, ctx.K = free, S, K
        return dyn, rep

    @staticmethod
    def backward(ctx, g_dyn, g_rep):
        post, prior, kl = ctx.saved_tensors
        rows = kl.numel()
        d_post = torch.empty_like(post) if ctx.needs_input_grad[0] else None
        d_prior = torch.empty_like(prior) if ctx.needs_input_grad[1] else None
        gd = g_dyn.contiguous() if g_dyn is not None else None
        gr = g_rep.contiguous() if g_rep is not None else None
        k.nat.call("sd_kl_bwd", k.p(post), k.p(prior), k.p(kl), k.p(gr), k.p(gd), float(ctx.free), k.p(d_post),
                   k.p(d_prior), rows, ctx.S, ctx.K, 0, 0, k.stream())
        return d_post, d_prior, None, None, None


class LossTermsFn(torch.autograd.Function):
    """The world-model loss dict and its weighted total (dreamer.py:571-576): term i = coefs[i] * mean(xs[i]), total =
    sum_i scales[i] * term_i in order. One launch forward (sd_loss_terms_fwd), one backward (every input's gradient,
    sd_loss_terms_bwd), instead of a reduce + scalar-op chain per term. Returns (total (), terms (n,))."""

    @staticmethod
    def forward(ctx, coefs, scales, *xs):
        xs = [x.contiguous() for x in xs]
        dev = xs[0].device
        terms = torch.empty(len(xs), dtype=torch.float32, device=dev)
        total = torch.empty(1, dtype=torch.float32, device=dev)
        k.loss_terms(xs, coefs, scales, terms, total)
        ctx.coefs, ctx.scales = list(coefs), list(scales)
        ctx.shapes = [x.shape for x in xs]
        ctx.dev = dev
        ctx.set_materialize_grads(False)  # an unused output's gradient stays None (no zeros launch)
        return total[0], terms

    @staticmethod
    def backward(ctx, g_total, g_terms):
        n = len(ctx.shapes)
        grads = [torch.empty(sh, dtype=torch.float32, device=ctx.dev) if ctx.needs_input_grad[2 + i] else None
                 for i, sh in enumerate(ctx.shapes)]
        if any(g is not None for g in grads):
            gt = g_total.reshape(1).contiguous() if g_total is not None else None
            gm = g_terms.contiguous() if g_terms is not None else None
            k.loss_terms_bwd([torch.Size(sh).numel() for sh in ctx.shapes], ctx.coefs, ctx.scales, grads, gt, gm)
        return (None, None) + tuple(grads[:n])


class TwoHotLogProbFn(torch.autograd.Function):
    """TwoHot.log_prob (distributions.py:100-129) for symexp bins; target detached."""

    @staticmethod
    def forward(ctx, logits, bins, target):
        NB = logits.shape[-1]
        l2 = _flat(logits).contiguous()
        t = target.reshape(-1).contiguous()
        out = torch.empty(l2.shape[0], dtype=torch.float32, device=logits.device)
        k.nat.call("sd_twohot_logp_fwd", k.p(l2), k.p(bins), k.p(t), k.p(out), l2.shape[0], NB, k.stream())
        ctx.save_for_backward(l2, bins, t)
        ctx.shape = logits.shape
        return out.view(logits.shape[:-1])

    @staticmethod
    def backward(ctx, g):
        l2, bins, t = ctx.saved_tensors
        dl = torch.empty_like(l2)
        k.nat.call("sd_twohot_logp_bwd", k.p(l2), k.p(bins), k.p(t), k.p(g.contiguous()), k.p(dl), l2.shape[0],
                   l2.shape[1], 0, k.stream())
        return dl.view(ctx.shape), None, None


class RepvalLossFn(torch.autograd.Function):
    """Replay-value loss mean(w * (-logp(ret) - logp(slow))) under the TwoHot value head (dreamer.py:652-658;
    TwoHot.log_prob distributions.py:100-129), w = 1 - is_last. The value head ran on every posterior step: logits
    (B, T, NB), slow / last (B, T); ret (B, T - 1) covers the first T - 1 steps (the reference's [:, :-1] slices are
    read in place). One launch for the row terms, one for their mean (K.device_mean), one backward launch for the
    logits gradient (both log-prob terms; zero on the last step). Targets and weights are detached."""

    @staticmethod
    def forward(ctx, logits, bins, ret, slow, last):
        B, Tl, NB = logits.shape
        Tr = ret.shape[1]
        l2, r, sl, la = logits.contiguous(), ret.contiguous(), slow.contiguous(), last.contiguous()
        rows = torch.empty(B * Tr, dtype=torch.float32, device=logits.device)
        k.nat.call("sd_repval_loss_fwd", k.p(l2), k.p(bins), k.p(r), k.p(sl), k.p(la), k.p(rows), B, Tl, Tr, NB,
                   k.stream())
        ctx.save_for_backward(l2, bins, r, sl, la)
        return k.device_mean(rows)

    @staticmethod
    def backward(ctx, g):
        l2, bins, r, sl, la = ctx.saved_tensors
        B, Tl, NB = l2.shape
        Tr = r.shape[1]
        dl = torch.empty_like(l2)
        gs = g.reshape(1).contiguous()
        k.nat.call("sd_repval_loss_bwd", k.p(l2), k.p(bins), k.p(r), k.p(sl), k.p(la), k.p(gs), 1.0 / (B * Tr),
                   k.p(dl), B, Tl, Tr, NB, k.stream())
        return dl, None, None, None, None


class ImagACLossFn(torch.autograd.Function):
    """Imagined policy and value losses (dreamer.py:623-636, 653-671) and their weighted sum: rows are the H * N
    time-major imagined steps; value logits vl (H*N, NB), logpi / ent (H*N) with gradients; ret (N, H), weight (N, H1),
    val (H1, N) time-major, slow (H, N), scale (device scalar) detached; sp / sv the loss scales. Forward: the row
    terms (sd_imag_ac_loss_fwd) and their means + the weighted total (one sd_loss_terms_fwd); backward: one launch
    from the total's gradient. Returns (total, policy, value, adv): adv (N, H) = (ret - val[:, :H]) / scale; only the
    total carries a gradient."""

    @staticmethod
    def forward(ctx, vl, logpi, ent, bins, ret, slow, weight, val, scale, coef, sp, sv):
        N, H = ret.shape
        H1 = weight.shape[1]
        NB = vl.shape[-1]
        l2 = _flat(vl).contiguous()
        lp, en = logpi.reshape(-1).contiguous(), ent.reshape(-1).contiguous()
        r, sl, w, v = ret.contiguous(), slow.reshape(-1).contiguous(), weight.contiguous(), val.contiguous()
        sc = scale.reshape(1).contiguous()
        rows = torch.empty(2, N * H, dtype=torch.float32, device=vl.device)
        adv = torch.empty(N, H, dtype=torch.float32, device=vl.device)
        k.nat.call("sd_imag_ac_loss_fwd", k.p(l2), k.p(bins), k.p(r), k.p(sl), k.p(w), k.p(v), k.p(sc), k.p(lp),
                   k.p(en), float(coef), N, H, H1, NB, k.p(rows[1]), k.p(rows[0]), k.p(adv), k.stream())
        means = torch.empty(2, dtype=torch.float32, device=vl.device)
        total = torch.empty(1, dtype=torch.float32, device=vl.device)
        k.loss_terms([rows[0], rows[1]], [1.0, 1.0], [sp, sv], means, total)  # policy, value; sp p + sv v
        ctx.save_for_backward(l2, bins, r, sl, w, adv)
        ctx.coef, ctx.sp, ctx.sv, ctx.shapes = float(coef), float(sp), float(sv), (vl.shape, logpi.shape, ent.shape)
        ctx.mark_non_differentiable(means, adv)
        ctx.set_materialize_grads(False)
        return total[0], means[0], means[1], adv

    @staticmethod
    def backward(ctx, g_total, _gp, _gv, _gadv):
        if _gp is not None or _gv is not None:  # (set_materialize_grads(False): unused outputs arrive as None)
            raise RuntimeError("ImagACLossFn: backpropagate the weighted total, not the policy / value loss alone")
        l2, bins, r, sl, w, adv = ctx.saved_tensors
        N, H = r.shape
        H1 = w.shape[1]
        vs, ls, es = ctx.shapes
        if g_total is None:
            return (None,) * 12
        dvl = torch.empty_like(l2)
        dlp = torch.empty(N * H, dtype=torch.float32, device=l2.device)
        den = torch.empty(N * H, dtype=torch.float32, device=l2.device)
        g = g_total.reshape(1).contiguous()
        k.nat.call("sd_imag_ac_loss_bwd", k.p(l2), k.p(bins), k.p(r), k.p(sl), k.p(w), k.p(adv), k.p(g), k.p(g),
                   ctx.sp, ctx.sv, ctx.coef, N, H, H1, l2.shape[1], k.p(dvl), k.p(dlp), k.p(den), k.stream())
        return dvl.view(vs), dlp.view(ls), den.view(es), None, None, None, None, None, None, None, None, None


class BernoulliLogProbFn(torch.autograd.Function):
    """Independent(Bernoulli(logits), 1).log_prob with a single logit (binary head, distributions.py:238)."""

    @staticmethod
    def forward(ctx, logit, value):
        l = logit.reshape(-1).contiguous()
        v = value.reshape(-1).contiguous().float()
        out = torch.empty_like(l)
        k.nat.call("sd_bernoulli_fwd", k.p(l), k.p(v), k.p(out), 0, l.numel(), k.stream())
        ctx.save_for_backward(l, v)
        ctx.shape = logit.shape
        return out.view(logit.shape[:-1])

    @staticmethod
    def backward(ctx, g):
        l, v = ctx.saved_tensors
        dl = torch.empty_like(l)
        k.nat.call("sd_bernoulli_bwd", k.p(l), k.p(v), k.p(g.contiguous()), k.p(dl), l.numel(), k.stream())
        return dl.view(ctx.shape), None


class BNormalLogProbEntFn(torch.autograd.Function):
    """bounded_normal (distributions.py:217-222): Independent(Normal(tanh(mean), std)).log_prob(a), .entropy()."""

    @staticmethod
    def forward(ctx, x, action, min_std, max_std):
        A = action.shape[-1]
        x2 = _flat(x).contiguous()
        a2 = _flat(action).contiguous()
        rows = x2.shape[0]
        lp = torch.empty(rows, dtype=torch.float32, device=x.device)
        ent = torch.empty_like(lp)
        k.nat.call("sd_bnormal_logp_ent_fwd", k.p(x2), k.p(a2), k.p(lp), k.p(ent), rows, A, float(min_std),
                   float(max_std), k.stream())
        ctx.save_for_backward(x2, a2)
        ctx.args = (A, min_std, max_std, x.shape)
        return lp.view(x.shape[:-1]), ent.view(x.shape[:-1])

    @staticmethod
    def backward(ctx, glp, gent):
        x2, a2 = ctx.saved_tensors
        A, mn, mx, shape = ctx.args
        dx = torch.empty_like(x2)
        k.nat.call("sd_bnormal_logp_ent_bwd", k.p(x2), k.p(a2), k.p(None if glp is None else glp.contiguous()),
                   k.p(None if gent is None else gent.contiguous()), k.p(dx), x2.shape[0], A, float(mn), float(mx),
                   k.stream())
        return dx.view(shape), None, None, None


class OneHotLogProbEntFn(torch.autograd.Function):
    """discrete actor OneHotDist (distributions.py:16-36): log_prob(one-hot action), entropy."""

    @staticmethod
    def forward(ctx, logits, action, unimix):
        K = logits.shape[-1]
        l2 = _flat(logits).contiguous()
        a2 = _flat(action).contiguous()
        rows = l2.shape[0]
        lp = torch.empty(rows, dtype=torch.float32, device=logits.device)
        ent = torch.empty_like(lp)
        k.nat.call("sd_onehot_logp_ent_fwd", k.p(l2), k.p(a2), k.p(lp), k.p(ent), rows, K, float(unimix), k.stream())
        ctx.save_for_backward(l2, a2)
        ctx.args = (K, unimix, logits.shape)
        return lp.view(logits.shape[:-1]), ent.view(logits.shape[:-1])

    @staticmethod
    def backward(ctx, glp, gent):
        l2, a2 = ctx.saved_tensors
        K, unimix, shape = ctx.args
        dl = torch.empty_like(l2)
        k.nat.call("sd_onehot_logp_ent_bwd", k.p(l2), k.p(a2), k.p(None if glp is None else glp.contiguous()),
                   k.p(None if gent is None else gent.contiguous()), k.p(dl), l2.shape[0], K, float(unimix),
                   k.stream())
        return dl.view(shape), None, None


class BarlowFn(torch.autograd.Function):
    """R2-Dreamer Barlow loss (dreamer.py:525-532) on x1 (N, E) (with grad) and x2 (N, E) (detached)."""

    @staticmethod
    def forward(ctx, x1, x2, lambd):
        x1, x2 = x1.contiguous(), x2.contiguous()
        Nr, E = x1.shape
        dev = x1.device
        m1, s1 = torch.empty(E, device=dev), torch.empty(E, device=dev)
        m2, s2 = torch.empty(E, device=dev), torch.empty(E, device=dev)
        k.nat.call("sd_colstats", k.p(x1), Nr, E, k.p(m1), k.p(s1), k.stream())
        k.nat.call("sd_colstats", k.p(x2), Nr, E, k.p(m2), k.p(s2), k.stream())
        n1 = torch.empty_like(x1)
        n2 = torch.empty_like(x2)
        k.nat.call("sd_standardize", k.p(x1), k.p(m1), k.p(s1), k.p(n1), Nr, E, 1e-8, k.stream())
        k.nat.call("sd_standardize", k.p(x2), k.p(m2), k.p(s2), k.p(n2), Nr, E, 1e-8, k.stream())
        c = k.mm(n1.t(), n2, alpha=1.0 / Nr)
        nb = 256
        part = torch.empty(2 * nb, device=dev)
        loss = torch.empty(1, device=dev)
        k.nat.call("sd_barlow_loss", k.p(c), E, float(lambd), k.p(part), nb, k.p(loss), k.stream())
        ctx.save_for_backward(x1, m1, s1, n2, c)
        ctx.lambd = lambd
        return loss[0]

    @staticmethod
    def backward(ctx, g):
        x1, m1, s1, n2, c = ctx.saved_tensors
        Nr, E = x1.shape
        dc = torch.empty_like(c)
        gg = g.reshape(1).contiguous()
        k.nat.call("sd_barlow_dc", k.p(c), k.p(gg), k.p(dc), E, float(ctx.lambd), k.stream())
        dn1 = k.mm(n2, dc.t(), alpha=1.0 / Nr)  # c = n1^T n2 / N  ->  dn1 = n2 dc^T / N
        dx1 = torch.empty_like(x1)
        k.nat.call("sd_standardize_bwd", k.p(x1), k.p(m1), k.p(s1), k.p(dn1), k.p(dx1), Nr, E, 1e-8, k.stream())
        return dx1, None, None


class MatmulNTFn(torch.autograd.Function):
    """a (M, K) @ b (N, K)^T with gradients for both operands on the HIP GEMM (DreamerPro's prototype scores,
    dreamer.py:801/811/832, where b is the normalised prototype table: a non-leaf, so its gradient is returned
    through autograd rather than accumulated into a parameter buffer)."""

    @staticmethod
    def forward(ctx, a, b):
        a, b = a.contiguous(), b.contiguous()
        ctx.save_for_backward(a, b)
        return k.mm(a, b.t())

    @staticmethod
    def backward(ctx, g):
        a, b = ctx.saved_tensors
        g = g.contiguous()
        da = k.mm(g, b, fast=True) if ctx.needs_input_grad[0] else None
        db = k.mm(g.t(), a, fast=True) if ctx.needs_input_grad[1] else None
        return da, db


class InfoNCEFn(torch.autograd.Function):
    """InfoNCE loss (dreamer.py:533-542): logits = x1 x2g^T (f32 GEMM), cross entropy against the diagonal; rows of x1
    (n, E) with grad, x2g (Nc, E) detached (all ranks' x2 under data parallel), row r labelled Nc-column r + off.
    Returns the mean over this rank's rows (the DP mean all-reduce of the gradients makes it the global mean)."""

    @staticmethod
    def forward(ctx, x1, x2g, off):
        x1 = x1.contiguous()
        n, nc = x1.shape[0], x2g.shape[0]
        logits = k.mm(x1, x2g.t())
        row = torch.empty(n, dtype=torch.float32, device=x1.device)
        lse = torch.empty(n, dtype=torch.float32, device=x1.device)
        loss = torch.empty(1, dtype=torch.float32, device=x1.device)
        k.nat.call("sd_infonce_fwd", k.p(logits), nc, n, nc, int(off), k.p(row), k.p(lse), k.p(loss), k.stream())
        ctx.save_for_backward(x2g, logits, lse)
        ctx.off = int(off)
        return loss[0]

    @staticmethod
    def backward(ctx, g):
        x2g, logits, lse = ctx.saved_tensors
        n, nc = logits.shape
        dl = torch.empty_like(logits)
        gg = g.reshape(1).contiguous()
        k.nat.call("sd_infonce_bwd", k.p(logits), nc, n, nc, ctx.off, k.p(lse), k.p(gg), 1.0 / n, k.p(dl), k.stream())
        return k.mm(dl, x2g, fast=True), None, None