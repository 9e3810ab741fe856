"""Per-kernel parity on the MI355X: every HIP op (forward and backward) vs the CPU oracle / torch fp32 restatement.

Tolerances: fp32 kernels with different summation order — max abs error scaled to the data (stated per test);
discrete outputs (latent indices) bit-exact except where the top-2 gumbel margin is below 1e-5.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import noise as nz
from oracle import ref_cpu as R

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _g(seed):
    return torch.Generator().manual_seed(seed)


def close(a, b, tol, what=""):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    err = (a - b).abs().max().item()
    scale = max(b.abs().max().item(), 1.0)
    assert err <= tol * scale, f"{what}: max abs err {err} (scale {scale})"


def test_noise_matches_oracle():
    from sdreamer import kernels as K
    g = K.fill_gumbel(4096, 1234, nz.STREAM_IMG, 3, offset=77).cpu().numpy()
    ref = nz.gumbel(1234, nz.STREAM_IMG, 3, np.arange(4096) + 77)
    assert np.abs(g - ref).max() <= 1e-6 * np.abs(ref).max()
    assert (g == ref).mean() > 0.999  # float64 transforms rounded once: bit-identical in practice
    n = K.fill_normal(4096, 99, nz.STREAM_ACT, 5).cpu().numpy()
    refn = nz.normal(99, nz.STREAM_ACT, 5, np.arange(4096))
    assert np.abs(n - refn).max() <= 1e-6


@pytest.mark.parametrize("same", [True, False])
def test_random_translate_bit_exact(same):
    """sd_random_translate vs oracle.ref_cpu.random_translate (nearest: the exact integer gather), with the shifts
    drawn from oracle/noise.aug_shifts at a nonzero slice-row offset (data-parallel shard of rows 5..)."""
    from sdreamer import kernels as K
    B, T, H, W, C, pad, seed, ro = 3, 4, 16, 12, 3, 3, 4242, 5
    img = torch.rand(B, T, H, W, C, generator=_g(3))
    out = K.random_translate(img.to(DEV), pad, seed, ro, same, bilinear=False).cpu()
    sh = torch.from_numpy(nz.aug_shifts(seed, B, ro, T, pad, same))
    assert torch.equal(out, R.random_translate(img, sh, pad, False))
    if same:
        assert (sh == sh[:, :1]).all()


@pytest.mark.parametrize("H,W,C,pad", [(64, 64, 3, 3), (64, 64, 3, 4), (9, 7, 2, 3), (32, 32, 1, 2)])
def test_random_translate_bilinear_matches_grid_sample(H, W, C, pad):
    """aug.bilinear (the config default): sd_random_translate restates F.grid_sample(bilinear, zeros, align_corners
    False) on the replicate-padded image with the reference's linspace grid + shift (dreamer.py:845-880); the
    oracle runs torch's own CPU grid_sample. Bit-exact, including the ~6e-8 neighbour weights of the float grid."""
    from sdreamer import kernels as K
    B, T, seed, ro = 4, 5, 777, 3
    img = (torch.randint(0, 256, (B, T, H, W, C), generator=_g(H + pad)).float() / 255.0)
    out = K.random_translate(img.to(DEV), pad, seed, ro, False, bilinear=True).cpu()
    sh = torch.from_numpy(nz.aug_shifts(seed, B, ro, T, pad, False))
    ref = R.random_translate(img, sh, pad, True)
    assert torch.equal(out, ref), (out - ref).abs().max()
    assert not torch.equal(ref, R.random_translate(img, sh, pad, False))  # the neighbour weights do mix in


@pytest.mark.parametrize("M,N", [(7, 256), (1024, 256), (33, 2048), (5, 4096), (100, 48), (64, 32), (3, 512)])
def test_rmsnorm_silu(M, N):
    from sdreamer import kernels as K
    x = torch.randn(M, N, generator=_g(M + N)) * 2
    w = 1 + 0.1 * torch.randn(N, generator=_g(1))
    dy = torch.randn(M, N, generator=_g(2))
    for act in (0, 1):
        xr, wr = x.clone().requires_grad_(), w.clone().requires_grad_()
        yr = R.rms(xr, wr)
        yr = F.silu(yr) if act else yr
        yr.backward(dy)
        y, rstd = K.rmsnorm_fwd(x.to(DEV), w.to(DEV), act=act)
        close(y, yr, 2e-6, "fwd")
        dw = torch.zeros(N, device=DEV)
        dx = K.rmsnorm_bwd(x.to(DEV), w.to(DEV), rstd, dy.to(DEV), act=act, dw=dw)
        close(dx, xr.grad, 1e-5, "dx")
        close(dw, wr.grad, 1e-5, "dw")


@pytest.mark.parametrize("K_,unimix", [(16, 0.01), (32, 0.01), (4, 0.01), (6, 0.01)])
def test_onehot_sample_fwd_bwd(K_, unimix):
    from sdreamer import kernels as K
    M, S = 257, 32 if K_ >= 16 else 1
    logits = torch.randn(M, S, K_, generator=_g(K_)) * 3
    seed, step, off = 4242, 7, 5
    st = K.onehot_sample(logits.to(DEV).contiguous(), K_, unimix, seed, nz.STREAM_IMG, step, off * S).cpu()
    g = torch.from_numpy(nz.gumbel_block(seed, nz.STREAM_IMG, step, M, off, S * K_)).view(M, S, K_)
    lr = logits.clone().requires_grad_()
    ref = R.st_gumbel_sample(R.unimix_logits(lr, unimix), g)
    # indices: exact except near-ties of the perturbed logits
    y = R.unimix_logits(logits, unimix) + g
    top2 = y.topk(2, -1).values
    margin = (top2[..., 0] - top2[..., 1])
    agree = st.argmax(-1) == ref.argmax(-1)
    assert bool(agree[margin > 1e-5].all())
    close(st, ref, 1e-6, "st value")
    dout = torch.randn(M, S, K_, generator=_g(3))
    ref.backward(dout)
    dl = K.onehot_sample_bwd(logits.to(DEV).contiguous(), dout.to(DEV), K_, unimix, seed, nz.STREAM_IMG, step, off * S)
    close(dl, lr.grad, 2e-5, "st grad")


def test_kl_fwd_bwd():
    from sdreamer import ops
    M, S, K_ = 300, 32, 16
    post = torch.randn(M, S * K_, generator=_g(1)) * 2
    prior = torch.randn(M, S * K_, generator=_g(2)) * 2
    pr, qr = post.clone().requires_grad_(), prior.clone().requires_grad_()
    rep = torch.clip(R.kl_cat(pr.view(M, S, K_), qr.detach().view(M, S, K_)).sum(-1), min=20.0)
    dyn = torch.clip(R.kl_cat(pr.detach().view(M, S, K_), qr.view(M, S, K_)).sum(-1), min=20.0)
    (0.1 * rep.mean() + dyn.mean()).backward()
    p, q = post.to(DEV).requires_grad_(), prior.to(DEV).requires_grad_()
    d, r = ops.KLFn.apply(p, q, 20.0, S, K_)
    close(d, dyn, 1e-5, "kl")
    (0.1 * r.mean() + d.mean()).backward()
    close(p.grad, pr.grad, 1e-5, "d post")
    close(q.grad, qr.grad, 1e-5, "d prior")


def test_twohot_mode_logp():
    from sdreamer import ops, kernels as K
    M = 513
    bins = R.twohot_bins(255)
    logits = -0.5 * (torch.arange(255) - 127).abs().float() + torch.randn(M, 255, generator=_g(5))
    target = torch.randn(M, generator=_g(6)) * 30
    target[:5] = torch.tensor([0.0, bins[3].item(), 1e9, -1e9, bins[200].item()])
    mode = K.twohot_mode(logits.to(DEV).contiguous(), bins.to(DEV)).cpu()
    close(mode, R.twohot_mode(logits, bins), 1e-5, "mode")
    lr = logits.clone().requires_grad_()
    lp = R.twohot_log_prob(lr, bins, target.unsqueeze(-1))
    gl = torch.randn(M, generator=_g(7))
    lp.backward(gl)
    l = logits.to(DEV).requires_grad_()
    out = ops.TwoHotLogProbFn.apply(l, bins.to(DEV), target.to(DEV))
    close(out, lp, 1e-5, "logp")
    out.backward(gl.to(DEV))
    close(l.grad, lr.grad, 1e-5, "dlogits")


def test_repval_loss_fused():
    """sd_repval_loss_fwd/bwd (ops.RepvalLossFn) vs the reference expression mean(w * (-logp(ret) - logp(slow)))
    (dreamer.py:652-658) on the oracle's TwoHot log-prob, w = 1 - is_last: the value logits / slow values / flags
    cover all T posterior steps and the loss reads the first T - 1 in place; the backward (seeded by a loss scale)
    leaves zeros on the last step."""
    from sdreamer import ops
    B, T = 16, 63
    bins = R.twohot_bins(255)
    logits = -0.5 * (torch.arange(255) - 127).abs().float() + torch.randn(B, T + 1, 255, generator=_g(11))
    ret = torch.randn(B, T, generator=_g(12)) * 30
    slow = torch.randn(B, T + 1, generator=_g(13)) * 30
    ret[0, :4] = torch.tensor([0.0, bins[3].item(), 1e9, -1e9])
    last = (torch.rand(B, T + 1, generator=_g(14)) < 0.1).float()
    scale = 0.3
    lr = logits.clone().requires_grad_()
    w = 1.0 - last[:, :-1]
    ref = torch.mean(w * (-R.twohot_log_prob(lr[:, :-1], bins, ret.unsqueeze(-1))
                          - R.twohot_log_prob(lr[:, :-1], bins, slow[:, :-1].unsqueeze(-1))))
    (ref * scale).backward()
    l = logits.to(DEV).requires_grad_()
    out = ops.RepvalLossFn.apply(l, bins.to(DEV), ret.to(DEV), slow.to(DEV), last.to(DEV))
    close(out, ref, 1e-5, "loss")
    torch.autograd.backward(out, torch.full((), scale, device=DEV))
    close(l.grad, lr.grad, 1e-5, "dlogits")
    assert (l.grad[:, -1] == 0).all()


def test_loss_terms_and_kl_clamp():
    """ops.LossTermsFn (sd_loss_terms_fwd/bwd): the loss dict's means and weighted total in one launch, gradients of
    every term in one launch; KLFn's clamped copies from the KL launch (torch.clamp(min=free), rssm.py:222-230)."""
    from sdreamer import ops
    xs = [torch.randn(16, 64, generator=_g(21)), torch.randn(1, generator=_g(22)), torch.randn(1024, generator=_g(23))]
    coefs, scales = [1.0, 1.0, -1.0], [0.5, 1.0, 2.0]
    xd = [x.to(DEV).requires_grad_() for x in xs]
    total, terms = ops.LossTermsFn.apply(coefs, scales, *xd)
    ref_terms = [c * x.mean() for c, x in zip(coefs, xs)]
    ref_total = sum(s * t for s, t in zip(scales, ref_terms))
    close(terms, torch.stack(ref_terms), 1e-6, "terms")
    close(total, ref_total, 1e-6, "total")
    torch.autograd.backward(total, torch.full((), 0.7, device=DEV))
    for x, xg, c, s in zip(xs, xd, coefs, scales):
        close(xg.grad, torch.full_like(x, 0.7 * s * c / x.numel()), 1e-6, "term grad")
    S, Kd, rows = 32, 16, 300
    post, prior = torch.randn(rows, S * Kd, generator=_g(24)), torch.randn(rows, S * Kd, generator=_g(25))
    dyn, rep = ops.KLFn.apply(post.to(DEV), prior.to(DEV), 1.0, S, Kd)
    from sdreamer import kernels as K
    raw = K.kl_rows(post.to(DEV), prior.to(DEV), S, Kd)
    assert torch.equal(dyn, torch.clamp(raw, min=1.0)) and torch.equal(rep, dyn)


def test_bnormal_and_bernoulli():
    from sdreamer import ops
    M, A = 300, 6
    x = torch.randn(M, 2 * A, generator=_g(1))
    a = torch.randn(M, A, generator=_g(2))
    xr = x.clone().requires_grad_()
    loc, sc = R.bounded_normal_params(xr, 0.1, 1.0)
    lp, ent = R.normal_log_prob(loc, sc, a), R.normal_entropy(sc)
    g1, g2 = torch.randn(M, generator=_g(3)), torch.randn(M, generator=_g(4))
    (lp * g1 + ent * g2).sum().backward()
    xd = x.to(DEV).requires_grad_()
    lpd, entd = ops.BNormalLogProbEntFn.apply(xd, a.to(DEV), 0.1, 1.0)
    close(lpd, lp, 1e-5, "logp")
    close(entd, ent, 1e-5, "ent")
    (lpd * g1.to(DEV) + entd * g2.to(DEV)).sum().backward()
    close(xd.grad, xr.grad, 1e-5, "dx")
    lo = torch.randn(M, 1, generator=_g(9)) * 3
    v = (torch.rand(M, 1, generator=_g(10)) > 0.3).float()
    lr_ = lo.clone().requires_grad_()
    ref = R.bernoulli_log_prob(lr_, v)
    ref.sum().backward()
    ld = lo.to(DEV).requires_grad_()
    out = ops.BernoulliLogProbFn.apply(ld, v.to(DEV))
    close(out, ref, 1e-6, "bern")
    out.sum().backward()
    close(ld.grad, lr_.grad, 1e-6, "bern grad")


def test_onehot_actor_logp_ent():
    from sdreamer import ops
    M, A = 200, 6
    lg = torch.randn(M, A, generator=_g(1))
    act = F.one_hot(torch.randint(0, A, (M,), generator=_g(2)), A).float()
    lr = lg.clone().requires_grad_()
    nl = R.unimix_logits(lr, 0.01)
    lp, ent = R.onehot_log_prob(nl, act), R.cat_entropy(nl)
    g1, g2 = torch.randn(M, generator=_g(3)), torch.randn(M, generator=_g(4))
    (lp * g1 + ent * g2).sum().backward()
    ld = lg.to(DEV).requires_grad_()
    a, b = ops.OneHotLogProbEntFn.apply(ld, act.to(DEV), 0.01)
    close(a, lp, 1e-5, "lp")
    close(b, ent, 1e-5, "ent")
    (a * g1.to(DEV) + b * g2.to(DEV)).sum().backward()
    close(ld.grad, lr.grad, 1e-5, "grad")


def test_gru_gates():
    from sdreamer import kernels as K
    M, G, Dg = 37, 8, 256
    D = G * Dg
    gates = torch.randn(M, 3 * D, generator=_g(1))
    h = torch.randn(M, D, generator=_g(2))
    gr, hr = gates.clone().requires_grad_(), h.clone().requires_grad_()
    r, c, u = (x.reshape(M, -1) for x in torch.chunk(gr.view(M, G, -1), 3, -1))
    r = torch.sigmoid(r)
    c = torch.tanh(r * c)
    u = torch.sigmoid(u - 1)
    out = u * c + (1 - u) * hr
    dy = torch.randn(M, D, generator=_g(3))
    out.backward(dy)
    o = K.gru_fwd(gates.to(DEV), h.to(DEV), G)
    close(o, out, 1e-6, "gru")
    dg, dh = K.gru_bwd(gates.to(DEV), h.to(DEV), dy.to(DEV), G)
    close(dg, gr.grad, 1e-6, "dgates")
    close(dh, hr.grad, 1e-6, "dh")


@pytest.mark.parametrize("ci,co,hw,nb", [(3, 32, 64, 3), (4, 32, 64, 3), (32, 48, 32, 2), (48, 64, 16, 4),
                                        (64, 64, 8, 5)])
def test_conv_pool_norm(ci, co, hw, nb):
    from sdreamer import ops
    x = torch.rand(nb, hw, hw, ci, generator=_g(ci)) - 0.5
    w = torch.randn(co, ci, 5, 5, generator=_g(co)) / (ci * 25) ** 0.5
    b = 0.1 * torch.randn(co, generator=_g(1))
    nw = 1 + 0.1 * torch.randn(co, generator=_g(2))
    xr = x.clone().requires_grad_()
    wr, br, nwr = w.clone().requires_grad_(), b.clone().requires_grad_(), nw.clone().requires_grad_()
    y = R.conv_same(xr.permute(0, 3, 1, 2), wr, br)
    y = F.silu(R.rms2d(F.max_pool2d(y, 2, 2), nwr))
    flat = y.reshape(nb, -1)  # NCHW flatten (networks.py:232)
    dy = torch.randn(flat.shape, generator=_g(3))
    flat.backward(dy)
    xd = x.to(DEV).requires_grad_()
    wd = w.permute(0, 2, 3, 1).contiguous().to(DEV)
    bd, nwd = b.to(DEV), nw.to(DEV)
    for t in (wd, bd, nwd):
        t.requires_grad_()
    out = ops.ConvPoolNormFn.apply(xd, wd, bd, nwd, True)
    close(out, flat, 2e-5, "fwd")
    out.backward(dy.to(DEV))
    close(xd.grad, xr.grad, 5e-5, "dx")
    close(wd.grad.permute(0, 3, 1, 2), wr.grad, 5e-5, "dw")
    close(bd.grad, br.grad, 5e-5, "db")
    close(nwd.grad, nwr.grad, 5e-5, "dnw")


@pytest.mark.parametrize("ci,co,hw,nb,nchw", [(4, 32, 64, 2, False), (32, 48, 32, 4, True), (48, 64, 16, 8, False),
                                             (64, 16, 8, 16, True), (16, 64, 8, 2, True)])
def test_conv_pool_fused_matches_two_launches(ci, co, hw, nb, nchw, monkeypatch):
    """sd_conv2d_fwd_pool vs sd_conv2d_fwd + sd_pool_rms_fwd: same k order (the implicit-GEMM kernels and the stage-2
    direct kernel), so the pooled values and argmax are bit-exact; rstd / y differ only in the channel-sum order
    (1e-6 relative). The 4-channel direct kernel (stage 1) contracts one tap per MFMA step instead of the 32-wide
    k tiles' interleave: pooled within 1e-6, argmax equal except on near-ties. (The f32 kernels: the bf16x6 direct
    kernel has its own test below.)"""
    from sdreamer import kernels as K
    monkeypatch.setattr(K, "CONV6", "")
    x = (torch.rand(nb, hw, hw, ci, generator=_g(ci)) - 0.5).to(DEV)
    w = (torch.randn(co, 5, 5, ci, generator=_g(co)) / (ci * 25) ** 0.5).to(DEV)
    b = (0.1 * torch.randn(co, generator=_g(1))).to(DEV)
    nw = (1 + 0.1 * torch.randn(co, generator=_g(2))).to(DEV)
    x[0, 1, 1, 0] = float("nan")  # NaN propagates through the max exactly like torch's max_pool2d
    fused = K.conv2d_fwd_pool(x, w, b, nw, nchw_flat=nchw)
    assert fused is not None, "shape should take the fused kernel"
    ref = K.pool_rms_fwd(K.conv2d_fwd(x, w, b), nw, nchw_flat=nchw)
    exact_order = ci != 4
    for a, r, what in zip(fused, ref, ("y", "pooled", "amax", "rstd")):
        if what == "amax":
            assert torch.equal(a, r) if exact_order else (a == r).float().mean().item() > 0.999, what
        elif what == "pooled" and exact_order:
            assert torch.equal(a.isnan(), r.isnan()) and torch.equal(a.nan_to_num(), r.nan_to_num()), what
        else:
            assert torch.equal(a.isnan(), r.isnan()), what
            close(a.nan_to_num(), r.nan_to_num(), 1e-6, what)


@pytest.mark.parametrize("nb", [3, 40])
def test_conv_pool_c4_grid_bit_identical(nb, monkeypatch):
    """Stage-1 direct kernel (conv_fwd_direct_pool_c4): every tile runs the same products in the same order whatever
    the grid, so the default one-round grid (SDHIP_C4_OCC resident workgroups per CU, 32 tiles each at the bench's
    1024 images), the round-5 grid (SDHIP_C4_TPW=16), a ragged 3 tiles per workgroup and a 3-per-CU round all give
    bit-identical outputs; nb = 3 leaves most workgroups of the default grid without a tile."""
    from sdreamer import kernels as K
    monkeypatch.setattr(K, "CONV6", "")
    x = (torch.rand(nb, 64, 64, 4, generator=_g(nb)) - 0.5).to(DEV)
    w = (torch.randn(32, 5, 5, 4, generator=_g(7)) / 10).to(DEV)
    b = (0.1 * torch.randn(32, generator=_g(1))).to(DEV)
    nw = (1 + 0.1 * torch.randn(32, generator=_g(2))).to(DEV)
    monkeypatch.delenv("SDHIP_C4_TPW", raising=False)
    monkeypatch.delenv("SDHIP_C4_OCC", raising=False)
    ref = [t.clone() for t in K.conv2d_fwd_pool(x, w, b, nw)]
    for env in ({"SDHIP_C4_TPW": "16"}, {"SDHIP_C4_TPW": "3"}, {"SDHIP_C4_TPW": "1"}, {"SDHIP_C4_OCC": "3"}):
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        out = K.conv2d_fwd_pool(x, w, b, nw)
        for a, r, what in zip(out, ref, ("y", "pooled", "amax", "rstd")):
            assert torch.equal(a, r), (env, what)
        for k in env:
            monkeypatch.delenv(k)


def test_upconv():
    from sdreamer import ops
    nb, hw, ci, co = 3, 8, 64, 48
    x = torch.randn(nb, hw, hw, ci, generator=_g(1))
    w = torch.randn(co, ci, 5, 5, generator=_g(2)) / (ci * 25) ** 0.5
    b = 0.1 * torch.randn(co, generator=_g(3))
    xr, wr, br = x.clone().requires_grad_(), w.clone().requires_grad_(), b.clone().requires_grad_()
    y = R.conv_same(F.interpolate(xr.permute(0, 3, 1, 2), scale_factor=2, mode="nearest"), wr, br).permute(0, 2, 3, 1)
    dy = torch.randn(y.shape, generator=_g(4))
    y.backward(dy)
    xd = x.to(DEV).requires_grad_()
    wd = w.permute(0, 2, 3, 1).contiguous().to(DEV).requires_grad_()
    bd = b.to(DEV).requires_grad_()
    out = ops.UpConvFn.apply(xd, wd, bd)
    close(out, y, 2e-5, "fwd")
    out.backward(dy.to(DEV))
    close(xd.grad, xr.grad, 5e-5, "dx")
    close(wd.grad.permute(0, 3, 1, 2), wr.grad, 5e-5, "dw")
    close(bd.grad, br.grad, 5e-5, "db")


def test_lambda_return_and_ema():
    from sdreamer import kernels as K
    N, T = 1024, 16
    rew = torch.randn(N, T, generator=_g(1))
    cl = torch.randn(N, T, generator=_g(2)) * 2
    val = torch.randn(N, T, generator=_g(3)) * 5
    cont = torch.sigmoid(cl)
    disc = 1 - 1 / 333
    ref = R.lambda_return(torch.zeros(N, T, 1), (1 - cont).unsqueeze(-1), rew.unsqueeze(-1), val.unsqueeze(-1),
                          val.unsqueeze(-1), disc, 0.95).squeeze(-1)
    wref = torch.cumprod(cont * disc, 1)
    co = torch.empty(N, T, device=DEV)
    wo = torch.empty(N, T, device=DEV)
    ret = K.lambda_return(rew.to(DEV), val.to(DEV), disc, 0.95, cont_logit=cl.to(DEV), cont_out=co, weight_out=wo)
    close(ret, ref, 1e-5, "ret")
    close(wo, wref, 1e-6, "weight")
    # time-major inputs read in place (sd_lambda_return_strided: the imagined heads' (T, N) outputs, the continue
    # logit a strided column of a wider logit matrix): bit-identical to the row-major call
    rew_tm, val_tm = rew.t().contiguous().to(DEV), val.t().contiguous().to(DEV)
    wide = torch.zeros(T * N, 3, device=DEV)
    wide[:, 1] = cl.t().reshape(-1).to(DEV)
    co2, wo2 = torch.empty(N, T, device=DEV), torch.empty(N, T, device=DEV)
    ret2 = K.lambda_return(rew_tm.t(), val_tm, disc, 0.95, cont_logit=wide[:, 1].view(T, N).t(), cont_out=co2,
                           weight_out=wo2, boot_row_stride=1, boot_t_stride=N)
    assert torch.equal(ret2, ret) and torch.equal(wo2, wo) and torch.equal(co2, co)
    ema = torch.tensor([0.3, 2.0])
    ema_d = ema.to(DEV)
    os_ = torch.empty(2, device=DEV)
    q = torch.empty(2, device=DEV)
    K.return_ema(ret.contiguous(), ema_d, os_, quantiles=q)
    qr = torch.quantile(ref.flatten(), torch.tensor([0.05, 0.95]))
    assert torch.equal(q.cpu(), qr), (q.cpu(), qr)  # exact order statistics + torch lerp
    er = ema.clone()
    off, sc = R.return_ema(er, ref)
    close(ema_d, er, 1e-7, "ema")
    close(os_, torch.stack([off, sc]), 1e-7, "offset/scale")


def test_barlow():
    from sdreamer import ops
    Nr, E = 256, 128
    x1 = torch.randn(Nr, E, generator=_g(1))
    x2 = torch.randn(Nr, E, generator=_g(2))
    xr = x1.clone().requires_grad_()
    x1n = (xr - xr.mean(0)) / (xr.std(0) + 1e-8)
    x2n = (x2 - x2.mean(0)) / (x2.std(0) + 1e-8)
    c = torch.mm(x1n.T, x2n) / Nr
    off = ~torch.eye(E, dtype=torch.bool)
    loss = (torch.diagonal(c) - 1).pow(2).sum() + 5e-4 * c[off].pow(2).sum()
    loss.backward()
    xd = x1.to(DEV).requires_grad_()
    ld = ops.BarlowFn.apply(xd, x2.to(DEV), 5e-4)
    close(ld, loss, 1e-5, "loss")
    ld.backward()
    close(xd.grad, xr.grad, 1e-5, "grad")


def test_metric_vector():
    """kernels.metric_vector (sd_multi_stats): mean / unbiased std / min / max of tensors above and below one chunk
    (SD_STAT_CHUNK), scalar tensors, scaled sums of several terms into one slot, and a mean taken as (mean - sub) / div
    with device scalars (the normalised-return metric), against torch."""
    from sdreamer import kernels as K
    g = _g(5)
    a = torch.randn(98304, generator=g) * 3 + 1
    b = torch.rand(15, 1024, generator=g)
    c = torch.tensor(2.5)
    d = torch.randn(7, generator=g)
    A, Bt, C, D = (t.to(DEV) for t in (a, b, c, d))
    vals = list(K.tensorstats(A, "a").values()) + list(K.tensorstats(Bt, "b").values()) + [
        C, K.Stat(D, K.STAT_STD), K.Stat(C) + K.Stat(A, scale=0.5) + K.Stat(D, K.STAT_MAX, scale=-2.0),
        K.Stat(Bt, sub=torch.tensor([0.25], device=DEV), div=torch.tensor([4.0], device=DEV))]
    got = K.metric_vector(vals).cpu().double()
    ref = torch.tensor([a.mean(), a.std(), a.min(), a.max(), b.mean(), b.std(), b.min(), b.max(), c, d.std(),
                        c + 0.5 * a.mean() - 2.0 * d.max(), ((b - 0.25) / 4.0).mean()]).double()
    assert torch.allclose(got, ref, rtol=2e-6, atol=1e-6), (got, ref)


def test_imag_ac_loss_fused():
    """ops.ImagACLossFn (sd_imag_ac_loss_fwd / _bwd + the weighted total) against the reference's torch formulation
    (dreamer.py:623-671 with TwoHot.log_prob, distributions.py:100-129): policy / value losses, their scaled sum, the
    advantage, and the gradients of logits, log-probs and entropies from the sum."""
    from sdreamer import ops
    from sdreamer.dreamer import _symexp_bins
    N, H, NB = 96, 5, 255
    H1 = H + 1
    g = _g(21)
    vl = torch.randn(H * N, NB, generator=g) * 0.5
    logpi = torch.randn(H * N, generator=g)
    ent = torch.rand(H * N, generator=g) + 0.5
    ret = torch.randn(N, H, generator=g) * 30
    slow = torch.randn(H, N, generator=g) * 30
    weight = torch.rand(N, H1, generator=g)
    val = torch.randn(N, H1, generator=g) * 30
    scale = torch.tensor(7.5)
    coef = 3e-4
    bins = _symexp_bins(NB, "cpu")
    vr, lr_, er = (t.clone().requires_grad_() for t in (vl, logpi, ent))
    adv = (ret - val[:, :H]) / scale
    w = weight[:, :H]
    pol = torch.mean(w * -(lr_.view(H, N).t() * adv + coef * er.view(H, N).t()))
    lt = R.twohot_log_prob(vr, bins, ret.t().reshape(-1))
    ls = R.twohot_log_prob(vr, bins, slow.reshape(-1))
    vlos = torch.mean(w * (-lt - ls).view(H, N).t())
    (2.0 * pol + 0.5 * vlos).backward()
    vd, ld, ed = (t.to(DEV).requires_grad_() for t in (vl, logpi, ent))
    t_, p_, v_, a_ = ops.ImagACLossFn.apply(vd, ld, ed, bins.to(DEV), ret.to(DEV), slow.to(DEV), weight.to(DEV),
                                            val.t().contiguous().to(DEV), scale.to(DEV), coef, 2.0, 0.5)  # time-major
    close(p_, pol, 1e-5, "policy")
    close(v_, vlos, 1e-5, "value")
    close(t_, 2.0 * pol + 0.5 * vlos, 1e-5, "weighted total")
    close(a_, adv, 1e-6, "adv")
    t_.backward()
    close(vd.grad, vr.grad, 1e-6, "d value logits")
    close(ld.grad, lr_.grad, 1e-6, "d logpi")
    close(ed.grad, er.grad, 1e-6, "d ent")


@pytest.mark.parametrize("Nr,E", [(512, 1024), (96, 64)])
def test_barlow_dist_steps(Nr, E):
    """parallel.BarlowSteps (the data-parallel Barlow's HIP launches, csrc/misc.hip sd_barlow_*) at world 1 against the
    single-GPU definition in torch fp32 (dreamer.py:525-532): loss and dx1 (x world = 1), and every intermediate the
    exchange steps pass on (sums, centred rows, q, c, stds, n2, z2) against its torch formula."""
    from sdreamer import parallel
    BS = parallel.BarlowSteps
    x1 = torch.randn(Nr, E, generator=_g(3)) * 2 + 0.5
    x2 = torch.randn(Nr, E, generator=_g(4)) - 0.25
    xr = x1.clone().requires_grad_()
    x1n = (xr - xr.mean(0)) / (xr.std(0) + 1e-8)
    x2n = (x2 - x2.mean(0)) / (x2.std(0) + 1e-8)
    c_ref = torch.mm(x1n.T, x2n) / Nr
    off = ~torch.eye(E, dtype=torch.bool)
    loss = (torch.diagonal(c_ref) - 1).pow(2).sum() + 5e-4 * c_ref[off].pow(2).sum()
    loss.backward()
    xd, x2d = x1.to(DEV), x2.to(DEV)
    Nt = float(Nr)
    sums = BS.colsums(xd, x2d)
    close(sums, torch.stack([x1.sum(0), x2.sum(0)]), 1e-5, "sums")
    d1, d2, stats = BS.center(xd, x2d, sums, Nt)
    m = sums.cpu() / Nt
    close(d1, x1 - m[0], 1e-6, "d1")
    close(d2, x2 - m[1], 1e-6, "d2")
    e1, e2 = x1 - m[0], x2 - m[1]
    close(stats[:2 * E], torch.cat([(e1 * e1).sum(0), (e2 * e2).sum(0)]), 1e-5, "q")
    close(stats[2 * E:].view(E, E), e1.t() @ e2, 1e-5, "d1^T d2")
    c, st, n2, z2 = BS.finish(stats, sums, Nt, d2)
    close(c, c_ref, 1e-5, "c")
    close(st, torch.stack([x1.std(0), x2.std(0)]), 1e-5, "stds")
    close(n2, x2n, 1e-5, "n2")
    close(z2, torch.zeros(E), 1e-4, "z2")
    xg = xd.clone().requires_grad_()
    ld = parallel._DistBarlowLoss.apply(xg, c, sums, st, n2, z2, 5e-4, Nt, 1)
    close(ld, loss, 1e-5, "loss")
    ld.backward()
    close(xg.grad, xr.grad, 1e-5, "dx1")


@pytest.mark.parametrize("Nr,E", [(512, 1024), (96, 64)])
def test_barlow_dist_steps_two_shards(Nr, E):
    """The sharded arithmetic of parallel.barlow_dist on the GPU launches, 2 ranks simulated in one process: each half
    of the rows runs colsums / center / finish / the loss backward with Nt = 2 R != R, the two all-reduces replaced
    by sums of the halves' tensors. Loss and c of every shard equal the full-batch torch fp32 definition
    (dreamer.py:525-532), and the ranks' dx1 rows (scaled by world) over world equal its gradient."""
    from sdreamer import parallel
    BS = parallel.BarlowSteps
    world, R = 2, Nr // 2
    x1 = torch.randn(Nr, E, generator=_g(5)) * 2 + 0.5
    x2 = torch.randn(Nr, E, generator=_g(6)) - 0.25
    xr = x1.clone().requires_grad_()
    x1n = (xr - xr.mean(0)) / (xr.std(0) + 1e-8)
    x2n = (x2 - x2.mean(0)) / (x2.std(0) + 1e-8)
    c_ref = torch.mm(x1n.T, x2n) / Nr
    off = ~torch.eye(E, dtype=torch.bool)
    loss = (torch.diagonal(c_ref) - 1).pow(2).sum() + 5e-4 * c_ref[off].pow(2).sum()
    loss.backward()
    Nt = float(Nr)
    shards = [(x1[r * R:(r + 1) * R].to(DEV), x2[r * R:(r + 1) * R].to(DEV)) for r in range(world)]
    sums = sum(BS.colsums(a, b) for a, b in shards)  # all-reduce 1
    cen = [BS.center(a, b, sums, Nt) for a, b in shards]
    stats = sum(s for _, _, s in cen)  # all-reduce 2
    dx = []
    for (a, _), (_, d2, _) in zip(shards, cen):
        c, st, n2, z2 = BS.finish(stats, sums, Nt, d2)
        close(c, c_ref, 1e-5, "c")
        close(n2, x2n[len(dx) * R:(len(dx) + 1) * R], 1e-5, "n2 rows")
        xg = a.clone().requires_grad_()
        ld = parallel._DistBarlowLoss.apply(xg, c, sums, st, n2, z2, 5e-4, Nt, world)
        close(ld, loss, 1e-5, "loss")
        ld.backward()
        dx.append(xg.grad)
    close(torch.cat(dx) / world, xr.grad, 1e-5, "dx1 (mean over ranks)")


@pytest.mark.parametrize("warmup", [1000, 0])
def test_laprop_agc_step(warmup):
    """sd_agc_laprop_step (AGC agc.py:15-53 + LaProp laprop.py:85-116 + LambdaLR warm-up dreamer.py:214-225) vs the
    oracle restatement, compared as per-element parameter DELTAS (|dp_gpu - dp_ref| <= 1e-4 |dp_ref| + 4 ulp(p))
    and moments (1e-5): a step of lr * O(1) = 4e-8 (warm-up) or 4e-5 is resolved, so a flipped sign, a skipped AGC
    clip (step 2 clips: 1000x larger gradients) or a wrong bias correction fails. Steps 1-3 mix unclipped and clipped
    tensors; the clip is active in step 2 only."""
    from sdreamer.optim import LaProp
    from oracle.ref_cpu import OracleAgent
    torch.manual_seed(0)
    shapes = [(256, 2560), (256,), (7, 5), (1000,)]
    ps_cpu = [torch.randn(s) for s in shapes]
    params = [torch.nn.Parameter(p.clone().to(DEV)) for p in ps_cpu]
    opt = LaProp(params, lr=4e-5, betas=(0.9, 0.999), eps=1e-20, agc=0.3, pmin=1e-3, warmup=warmup)

    class _S:
        pass
    ag = OracleAgent.__new__(OracleAgent)
    ag.P = {str(i): p.clone().requires_grad_() for i, p in enumerate(ps_cpu)}
    ag.s = _S()
    ag.s.shapes = {str(i): s for i, s in enumerate(shapes)}
    ag.lr0, ag.warmup, ag.betas, ag.eps, ag.agc, ag.pmin = 4e-5, warmup, (0.9, 0.999), 1e-20, 0.3, 1e-3
    ag.opt_step, ag.state = 0, {}
    for it in range(3):
        grads = [torch.randn(s) * (10.0 if it == 1 else 0.01) for s in shapes]
        prev_g = [p.data.detach().cpu().double() for p in params]
        prev_r = [ag.P[str(i)].data.clone().double() for i in range(len(shapes))]
        for i, g in enumerate(grads):
            params[i].grad.copy_(g.to(DEV))
            ag.P[str(i)].grad = g.clone()
        opt.step()
        ag.agc_()
        ag.laprop_step()
        ag.opt_step += 1
        sd = opt.state_dict()["state"]
        for i in range(len(shapes)):
            pr = ag.P[str(i)].data
            d_got = params[i].data.detach().cpu().double() - prev_g[i]
            d_ref = pr.double() - prev_r[i]
            tol = 1e-4 * d_ref.abs() + 4 * torch.from_numpy(np.spacing(np.abs(pr.numpy()))).double()
            assert ((d_got - d_ref).abs() <= tol).all(), (i, it, float((d_got - d_ref).abs().max()))
            st = ag.state[id(ag.P[str(i)])]
            for nm in ("exp_avg", "exp_avg_sq"):
                a, b = sd[i][nm].cpu().double(), st[nm].double()
                assert ((a - b).abs() <= 1e-5 * b.abs() + 1e-5 * b.abs().max()).all(), (nm, i, it, float((a - b).abs().max()))
            assert abs(sd[i]["exp_avg_lr_1"] - st["exp_avg_lr_1"]) <= 1e-12 * abs(st["exp_avg_lr_1"])


def test_laprop_grad_scale_and_gate():
    """The fused step's data-parallel mean (grad_scale = 1 / world after a sum all-reduce) and tensor gate (DreamerPro's
    prototype freeze) equal the ATen forms they replace, bit for bit: grads g * world with grad_scale 1 / world (world a
    power of two) == g; gate 0 == a zeroed gradient, gate 1 == the gradient."""
    from sdreamer.optim import LaProp
    shapes = [(64, 96), (96,), (33, 7)]
    g0 = [torch.randn(s, generator=_g(31 + i)) for i, s in enumerate(shapes)]
    p0 = [torch.randn(s, generator=_g(41 + i)) for i, s in enumerate(shapes)]

    def run(scale, gate_val, gmul, zero_gated):
        params = [torch.nn.Parameter(p.clone().to(DEV)) for p in p0]
        opt = LaProp(params, lr=4e-5, warmup=0)
        opt.grad_scale = scale
        gate = torch.full((1,), 1.0 if gate_val is None else gate_val, device=DEV)
        if gate_val is not None:
            opt.gate = (1, gate)
        for it in range(2):
            for i, g in enumerate(g0):
                gg = g * gmul * (it + 1)
                params[i].grad.copy_(torch.zeros_like(gg) if (zero_gated and i == 1) else gg.to(DEV))
            opt.step()
        return [p.detach().cpu() for p in params]

    ref = run(1.0, None, 1.0, False)
    for got in (run(0.125, None, 8.0, False), run(1.0, 1.0, 1.0, False)):
        assert all(torch.equal(a, b) for a, b in zip(got, ref))
    gated = run(1.0, 0.0, 1.0, False)
    zeroed = run(1.0, None, 1.0, True)
    assert all(torch.equal(a, b) for a, b in zip(gated, zeroed))
    # zero_grads_after (graph-replayed updates: zero_grad folded into the step): the same parameters, every gradient 0
    params = [torch.nn.Parameter(p.clone().to(DEV)) for p in p0]
    opt = LaProp(params, lr=4e-5, warmup=0)
    opt.zero_grads_after = True
    for it in range(2):
        for i, g in enumerate(g0):
            params[i].grad.add_(g.to(DEV) * (it + 1))  # accumulates onto the zeros the previous step left
        opt.step()
    assert all(torch.equal(a.detach().cpu(), b) for a, b in zip(params, ref))
    assert not opt.arena.grad.any()


def test_polyak():
    """sd_polyak = the slow-critic update s = 0.02 v + 0.98 s (dreamer.py:242-249), within 1 ulp of the torch f32
    expression (fma contraction)."""
    from sdreamer import _native as nat, kernels as K
    g = torch.Generator().manual_seed(3)
    v = torch.randn(100003, generator=g)
    s0 = torch.randn(100003, generator=g)
    dst = s0.clone().to(DEV)
    nat.call("sd_polyak", K.p(v.to(DEV)), K.p(dst), v.numel(), 0.02, K.stream())
    ref = (0.02 * v + (1 - 0.02) * s0)
    assert ((dst.cpu() - ref).abs() <= torch.from_numpy(np.spacing(np.abs(ref.numpy())))).all()


@pytest.mark.parametrize("ci,co,hw,nb", [(4, 32, 64, 3), (32, 48, 32, 8), (48, 64, 16, 16), (64, 64, 8, 40),
                                        (16, 32, 16, 2), (64, 16, 32, 1)])
def test_conv_backward_bf16x3(ci, co, hw, nb):
    """Split-bf16 conv backward (sd_conv2d_dgrad_bf16x3 / sd_conv2d_wgrad_bf16x3) vs the f32 kernels:
    |err| <= 4e-5 * (the same contraction on |operands|) elementwise (per-product split error <= 3 * 2^-17)."""
    from sdreamer import kernels as K
    x = (torch.rand(nb, hw, hw, ci, generator=_g(ci + hw)) - 0.5).to(DEV)
    w = (torch.randn(co, 5, 5, ci, generator=_g(co)) / (ci * 25) ** 0.5).to(DEV)
    dy = torch.randn(nb, hw, hw, co, generator=_g(7)).to(DEV)
    dx = K.conv2d_dgrad(dy, w, fast=True)
    dx_ref = K.conv2d_dgrad(dy, w, fast=False)
    bound = 4e-5 * K.conv2d_dgrad(dy.abs(), w.abs(), fast=False) + 1e-6
    assert ((dx - dx_ref).abs() - bound).max().item() <= 0, "dgrad"
    if ci in (16, 32, 48, 64):  # the split kernel's output-channel tiles; other widths take the f32 kernel
        assert (dx - dx_ref).abs().max().item() > 0, "dgrad took the f32 path"
    dw = K.conv2d_wgrad(x, dy, 5, 5, fast=True)
    dw_ref = K.conv2d_wgrad(x, dy, 5, 5, fast=False)
    bound = 4e-5 * K.conv2d_wgrad(x.abs(), dy.abs(), 5, 5, fast=False) + 1e-5
    assert ((dw - dw_ref).abs() - bound).max().item() <= 0, "wgrad"
    if K.nat.fns["sd_conv2d_wgrad_bf16x3_slabs"](nb, hw, hw, ci, co, 5, 5, 0) > 0:  # the split kernel's range
        assert (dw - dw_ref).abs().max().item() > 0, "wgrad took the f32 path"


@pytest.mark.parametrize("ci,co,hw,nb,nchw", [(32, 48, 32, 4, False), (48, 64, 16, 8, True), (48, 64, 16, 1, False)])
def test_conv_pool_bf16x6_matches_f32(ci, co, hw, nb, nchw, monkeypatch):
    """The encoder stage forward on the three-way split-bf16 direct kernel (sd_conv2d_fwd_pool6) against the exact
    f32 kernel: an fp32-accurate contraction (each product's dropped terms <= 2^-26 |ab|), so the conv outputs agree
    to fp32 rounding: |pooled - ref| <= 2e-6 * (the same contraction on |x|, |w|) + 1e-7; argmax equal except where
    the window's top two conv outputs are that close; NaN inputs propagate the same way."""
    from sdreamer import kernels as K
    x = (torch.rand(nb, hw, hw, ci, generator=_g(ci)) - 0.5).to(DEV)
    w = (torch.randn(co, 5, 5, ci, generator=_g(co)) / (ci * 25) ** 0.5).to(DEV)
    b = (0.1 * torch.randn(co, generator=_g(1))).to(DEV)
    nw = (1 + 0.1 * torch.randn(co, generator=_g(2))).to(DEV)
    x[0, 1, 1, 0] = float("nan")
    monkeypatch.setattr(K, "CONV6", "1")
    six = K.conv2d_fwd_pool(x, w, b, nw, nchw_flat=nchw)
    monkeypatch.setattr(K, "CONV6", "")
    ref = K.conv2d_fwd_pool(x, w, b, nw, nchw_flat=nchw)
    conv_abs = K.conv2d_fwd(x.abs().nan_to_num(), w.abs(), None)  # (nb, hw, hw, co) bound operand
    bound = 2e-6 * F.max_pool2d(conv_abs.permute(0, 3, 1, 2), 2, 2).permute(0, 2, 3, 1) + 1e-7
    y6, p6, a6, r6 = six
    yr, pr, ar, rr = ref
    assert torch.equal(p6.isnan(), pr.isnan()) and torch.equal(y6.isnan(), yr.isnan())
    assert ((p6 - pr).nan_to_num().abs() - bound).max().item() <= 0, "pooled"
    assert (p6 - pr).nan_to_num().abs().max().item() > 0, "pool6 took the f32 path"
    assert (a6 == ar).float().mean().item() > 0.999, "amax"
    close(r6.nan_to_num(), rr.nan_to_num(), 1e-5, "rstd")
    close(y6.nan_to_num(), yr.nan_to_num(), 1e-5, "y")


@pytest.mark.parametrize("ci,co,hw,nb,nchw", [(32, 48, 32, 4, False), (32, 48, 32, 3, True), (48, 64, 16, 5, True),
                                               (48, 64, 16, 2, False)])
def test_conv_pool_bf16x6_ring_bit_identical(ci, co, hw, nb, nchw, monkeypatch):
    """The bf16x6 stage forward with the weight through the LDS ring (conv_fwd6r_direct_pool: the 32 -> 48 stage on
    512-pixel tiles with 64 pixels per wave, or 256 / 32 (SDHIP_CONV6_MT=2); the 48 -> 64 stage on 256-pixel tiles and
    the channel-group-major patch) against the per-lane-weight kernel (SDHIP_CONV6_RING=0, 128-pixel tiles), one tile or
    several per workgroup, with or without the fragment pipeline: the same products in the same k order, so every
    output is bit-identical."""
    from sdreamer import kernels as K
    x = (torch.rand(nb, hw, hw, ci, generator=_g(21)) - 0.5).to(DEV)
    w = (torch.randn(co, 5, 5, ci, generator=_g(22)) / (ci * 25) ** 0.5).to(DEV)
    b = (0.1 * torch.randn(co, generator=_g(23))).to(DEV)
    nw = (1 + 0.1 * torch.randn(co, generator=_g(24))).to(DEV)
    monkeypatch.setattr(K, "CONV6", "1")
    rings = [K.conv2d_fwd_pool(x, w, b, nw, nchw_flat=nchw)]
    for tpw in ("3", "16"):  # multi-tile workgroups (the bench's default), ragged tile ranges, idle workgroups
        monkeypatch.setenv("SDHIP_CONV6_TPW", tpw)
        rings.append(K.conv2d_fwd_pool(x, w, b, nw, nchw_flat=nchw))
    monkeypatch.setenv("SDHIP_CONV6_MT", "2")  # (32 -> 48: 256-pixel tiles, 32 pixels per wave; default 4: 512, 64)
    for tpw in ("1", "3"):
        monkeypatch.setenv("SDHIP_CONV6_TPW", tpw)
        rings.append(K.conv2d_fwd_pool(x, w, b, nw, nchw_flat=nchw))
    monkeypatch.delenv("SDHIP_CONV6_MT")
    monkeypatch.delenv("SDHIP_CONV6_TPW")
    monkeypatch.setenv("SDHIP_CONV6_PIPE", "1")
    rings.append(K.conv2d_fwd_pool(x, w, b, nw, nchw_flat=nchw))
    monkeypatch.delenv("SDHIP_CONV6_PIPE")
    monkeypatch.setenv("SDHIP_CONV6_RING", "0")
    lane = K.conv2d_fwd_pool(x, w, b, nw, nchw_flat=nchw)
    for ring in rings:
        for a, r, what in zip(ring, lane, ("y", "pooled", "amax", "rstd")):
            assert torch.equal(a, r), what


@pytest.mark.parametrize("cd,ci,hw,nb", [(48, 32, 32, 8), (64, 48, 16, 16), (48, 32, 32, 1)])
def test_conv_dgrad_direct_matches_implicit_gemm(cd, ci, hw, nb, monkeypatch):
    """The direct bwd-data kernel (sd_conv2d_dgrad_direct: dOut patch staged once per workgroup; the 48 -> 32 stage on
    512-pixel tiles of 64-pixel waves and the 64 -> 48 one on whole-image tiles of 64-pixel waves, or both on 128-pixel
    tiles of 32-pixel waves with SDHIP_DGRAD_MT=2 / SDHIP_DGRAD3_MT=2) against the implicit-GEMM one
    (sd_conv2d_dgrad_bf16x3): the same (hi, lo) splits, the same three products per k and the same k order, so bit for
    bit the same dIn; and both within the split-bf16 bound of the f32 kernel."""
    from sdreamer import kernels as K
    w = (torch.randn(cd, 5, 5, ci, generator=_g(cd + ci)) / (ci * 25) ** 0.5).to(DEV)
    dy = torch.randn(nb, hw, hw, cd, generator=_g(hw)).to(DEV)
    wf = K.conv_flip_weight(w)
    ws = K.conv_split_weight(wf)
    dx = torch.empty(nb, hw, hw, ci, device=DEV)
    assert K.nat.call_shaped("sd_conv2d_dgrad_direct", K.p(dy), K.p(ws), K.p(dx), nb, hw, hw, cd, ci, 5, 5, 2,
                             K.stream()), "direct kernel not instantiated for this shape"
    dx_gemm = K.conv2d_dgrad(dy, w, fast=True, direct=False)
    assert torch.equal(dx, dx_gemm)
    for knob, val in (("SDHIP_DGRAD_MT", "2"), ("SDHIP_DGRAD3_MT", "2")):  # (each applies to one stage)
        monkeypatch.setenv(knob, val)
        dx2 = torch.empty_like(dx)
        assert K.nat.call_shaped("sd_conv2d_dgrad_direct", K.p(dy), K.p(ws), K.p(dx2), nb, hw, hw, cd, ci, 5, 5, 2,
                                 K.stream())
        monkeypatch.delenv(knob)
        assert torch.equal(dx2, dx_gemm), knob
    dx_ref = K.conv2d_dgrad(dy, w, fast=False)
    bound = 4e-5 * K.conv2d_dgrad(dy.abs(), w.abs(), fast=False) + 1e-6
    assert ((dx - dx_ref).abs() - bound).max().item() <= 0


@pytest.mark.parametrize("ci,co,hw,nb", [(4, 32, 64, 3), (32, 48, 32, 2)])
def test_first_stage_pooled_wgrad_reordered_sums(ci, co, hw, nb):
    """A stage without input gradient (the encoder's first) takes the compact backward — sd_pool_rms_bwd_compact +
    sd_conv2d_wgrad_pool, the conv gradient expanded from (pooled gradient, argmax) inside the direct kernel — and
    must give the dense path's weight / bias / norm gradients: the same values staged, in 512-pixel row blocks (the
    dense direct kernel stages 128) — so the f32 sums are reordered (close at 2e-5) and the norm gradient is exact."""
    from sdreamer import kernels as K
    from sdreamer import ops
    x = torch.rand(nb, hw, hw, ci, generator=_g(5)).to(DEV)
    grads = []
    for compact in (True, False):
        w = (torch.randn(co, 5, 5, ci, generator=_g(6)) / (ci * 25) ** 0.5).to(DEV).requires_grad_()
        b = (0.1 * torch.randn(co, generator=_g(7))).to(DEV).requires_grad_()
        nw = (1 + 0.1 * torch.randn(co, generator=_g(8))).to(DEV).requires_grad_()
        ops.POOL_COMPACT = compact
        try:
            y = ops.ConvPoolNormFn.apply(x, w, b, nw, False)
            gy = torch.randn(y.shape, generator=_g(9)).to(DEV)
            y.backward(gy)
        finally:
            ops.POOL_COMPACT = True
        grads.append((w.grad.clone(), b.grad.clone(), nw.grad.clone()))
    if K.conv2d_wgrad_pool_slabs(x, co, 5, 5) > 0 and ci == 4:
        assert torch.equal(grads[0][2], grads[1][2]), "nw"
        for a, r, what in zip(grads[0][:2], grads[1][:2], ("w", "b")):
            close(a, r, 2e-5, what)
    else:
        for a, r, what in zip(grads[0], grads[1], ("w", "b", "nw")):
            close(a, r, 2e-5, what)


@pytest.mark.parametrize("nb", [3, 16])
def test_first_stage_pooled_wgrad_bf16x3(nb, monkeypatch):
    """sd_conv2d_wgrad_pool_bf16x3 (the first stage's bwd-weight on the split-bf16 direct kernel, pooled gradient routed
    through the argmax while staged, 32-pixel steps dealt to the 8 waves) against the f32 pooled kernel on the same
    (pooled gradient, argmax): the weight / bias gradients within the split-bf16 bound 4e-5 * sum |dy| |x| per element
    (the bound the dense split-bf16 bwd-weight meets), the norm gradient (not a contraction) exact."""
    from sdreamer import kernels as K
    from sdreamer import ops
    ci, co, hw = 4, 32, 64
    x = torch.rand(nb, hw, hw, ci, generator=_g(15)).to(DEV) - 0.5
    x[..., 3] = 0.0  # the padded fourth channel, as the encoder feeds it
    if K.nat.fns["sd_conv2d_wgrad_pool_bf16x3_slabs"](nb, hw, hw, ci, co, 5, 5) <= 0:
        pytest.skip("shape outside the split-bf16 pooled kernel")
    grads = []
    for x3 in (True, False):
        monkeypatch.setattr(K, "WGRAD1_X3", x3)
        w = (torch.randn(co, 5, 5, ci, generator=_g(16)) / (ci * 25) ** 0.5).to(DEV).requires_grad_()
        b = (0.1 * torch.randn(co, generator=_g(17))).to(DEV).requires_grad_()
        nw = (1 + 0.1 * torch.randn(co, generator=_g(18))).to(DEV).requires_grad_()
        y = ops.ConvPoolNormFn.apply(x, w, b, nw, False)
        gy = torch.randn(y.shape, generator=_g(19)).to(DEV)
        y.backward(gy)
        grads.append((w.grad.clone(), b.grad.clone(), nw.grad.clone()))
        if not x3:  # the bound: the same contraction on |dy| and |x|, from the dense f32 path's expanded gradient
            _, pooled, amax, rstd = K.conv2d_fwd_pool(x.contiguous(), w.detach(), b.detach(), nw.detach())
            dconv = K.pool_rms_bwd(pooled, amax, nw.detach(), rstd, gy, hw, hw, torch.zeros_like(nw))
            absw = K.conv2d_wgrad(x.abs(), dconv.abs(), 5, 5, fast=False)
    assert torch.equal(grads[0][2], grads[1][2]), "nw"
    bound = 4e-5 * absw + 1e-6
    got = torch.cat([grads[0][0].reshape(co, -1), grads[0][1][:, None]], 1)
    ref = torch.cat([grads[1][0].reshape(co, -1), grads[1][1][:, None]], 1)
    assert ((got - ref).abs() - bound).max().item() <= 0, float(((got - ref).abs() / bound).max())


def test_layout_copies_exact():
    """sd_layout_copies_run (the scan backward's W^T images, the conv pad, get_feat's strided concat): transposes of
    batched, ragged (not multiple of 64 / 4), strided and misaligned sources and column pads into a strided slot,
    all in one launch, must equal torch's copies bit for bit."""
    from sdreamer import kernels as K
    g = _g(11)
    ents, want = [], []
    for nb, rows, cols, sr_pad, off in [(1, 2048, 256, 0, 0), (8, 256, 512, 0, 0), (3, 70, 45, 3, 1),
                                        (1, 5, 130, 0, 0), (2, 129, 64, 4, 0), (1, 1, 1, 0, 0), (1, 64, 7, 1, 2)]:
        base = torch.randn(nb * rows * (cols + sr_pad) + off, generator=g).to(DEV)
        src = base[off:].view(nb, rows, cols + sr_pad)[:, :, :cols]
        dst = torch.full((nb, cols, rows), float("nan"), device=DEV)
        ents.append((src, dst, nb, rows, cols, src.stride(0), src.stride(1), cols, 0))
        want.append((dst, src.transpose(1, 2)))
    x = torch.randn(33, 5, generator=g).to(DEV)
    slot = torch.full((33, 12), float("nan"), device=DEV)
    ents.append((x, slot, 1, 33, 5, 0, 5, 9, 1, 12))
    ref = torch.cat([x, torch.zeros(33, 4, device=DEV)], 1)
    K.layout_copies(ents)
    torch.cuda.synchronize()
    for i, (d, r) in enumerate(want):
        assert torch.equal(d, r.contiguous()), f"entry {i}"
    assert torch.equal(slot[:, :9], ref)
    assert torch.isnan(slot[:, 9:]).all()
