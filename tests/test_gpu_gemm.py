"""GEMM kernel (sd_gemm_f32) vs torch fp32 reference, all operand layouts, batching, split-K, bias/beta."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def _ref(a, b, bias=None, c=None, alpha=1.0, beta=0.0):
    r = alpha * (a.double() @ b.double())
    if bias is not None:
        r = r + bias.double()
    if c is not None and beta != 0:
        r = r + beta * c.double()
    return r


@pytest.mark.parametrize("M,N,K", [(1, 1, 1), (16, 256, 2048), (37, 53, 71), (1024, 256, 2560), (300, 129, 1000),
                                   (64, 2048, 768), (4096, 64, 1600)])
@pytest.mark.parametrize("ak", [True, False])
@pytest.mark.parametrize("bk", [True, False])
def test_gemm_layouts(M, N, K, ak, bk):
    from sdreamer import kernels as k
    dev = "cuda"
    g = torch.Generator(device="cpu").manual_seed(M * 7 + N * 3 + K)
    a0 = torch.randn(M, K, generator=g).to(dev)
    b0 = torch.randn(K, N, generator=g).to(dev)
    a = a0 if ak else a0.t().contiguous().t()
    b = b0.t().contiguous().t() if bk else b0
    bias = torch.randn(N, generator=g).to(dev)
    out = k.mm(a, b, bias=bias)
    ref = _ref(a0, b0, bias)
    err = (out.double() - ref).abs().max().item()
    scale = (a0.double().abs() @ b0.double().abs()).max().item() + 1
    assert err <= 2e-6 * scale, err


@pytest.mark.parametrize("M,N,K", [(16, 256, 2048), (16, 2048, 768), (1, 255, 256), (32, 512, 256), (16, 6, 2560),
                                   (3, 100, 77)])
@pytest.mark.parametrize("bk", [True, False])
def test_gemm_skinny(M, N, K, bk):
    from sdreamer import kernels as k
    g = torch.Generator(device="cpu").manual_seed(M + N + K)
    a = torch.randn(M, K, generator=g).to("cuda")
    w = torch.randn(N, K, generator=g).to("cuda")
    b = w.t() if bk else w.t().contiguous()
    bias = torch.randn(N, generator=g).to("cuda")
    c0 = torch.randn(M, N, generator=g).to("cuda")
    out = c0.clone()
    k.gemm(a, b, out, bias=bias, beta=1.0)
    ref = a.double() @ w.double().t() + bias.double() + c0.double()
    assert (out.double() - ref).abs().max().item() < 2e-6 * (a.abs().double() @ w.abs().double().t()).max().item() + 1e-5


def test_colsum_long():
    from sdreamer import kernels as k
    g = torch.Generator(device="cpu").manual_seed(3)
    x = torch.randn(20000, 255, generator=g).to("cuda")
    out = torch.ones(255, device="cuda")
    k.colsum(x, out, accumulate=True)
    assert (out.double().cpu() - (x.double().sum(0).cpu() + 1)).abs().max().item() < 1e-3


@pytest.mark.parametrize("ks", [1, 3, 8])
def test_gemm_splitk_beta_batched(ks):
    from sdreamer import kernels as k
    dev = "cuda"
    g = torch.Generator(device="cpu").manual_seed(5)
    Bt, M, N, K = 8, 16, 256, 1024
    a = torch.randn(M, Bt * K, generator=g).to(dev)  # BlockLinear-style: block views of one row-major input
    w = torch.randn(Bt, N, K, generator=g).to(dev)
    av = a.view(M, Bt, K).permute(1, 0, 2)  # (Bt, M, K) strided
    bv = w.transpose(1, 2)  # (Bt, K, N), k contiguous
    c0 = torch.randn(M, Bt * N, generator=g).to(dev)
    out = c0.clone()
    ov = out.view(M, Bt, N).permute(1, 0, 2)
    k.gemm(av, bv, ov, alpha=0.5, beta=1.0, ksplit=ks)
    ref = 0.5 * torch.einsum("mbk,bnk->mbn", a.view(M, Bt, K).double(), w.double()).reshape(M, Bt * N) + c0.double()
    assert (out.double() - ref).abs().max().item() < 1e-3


@pytest.mark.parametrize("M,N,K", [(64, 64, 64), (1024, 256, 2560), (300, 129, 1000), (15360, 256, 2560),
                                   (256, 2560, 15360), (2048, 1024, 512), (4096, 65, 1600), (100, 200, 3000)])
@pytest.mark.parametrize("ak", [True, False])
@pytest.mark.parametrize("bk", [True, False])
def test_gemm_bf16x3_layouts(M, N, K, ak, bk):
    """Split-bf16 path: |err_ij| <= 4e-5 * sum_k |a_ik||b_kj| (per-product split error <= 3 * 2^-17, f32 sums)."""
    from sdreamer import kernels as k
    dev = "cuda"
    g = torch.Generator(device="cpu").manual_seed(M * 5 + N * 3 + K)
    a0 = torch.randn(M, K, generator=g).to(dev)
    b0 = torch.randn(K, N, generator=g).to(dev)
    a = a0 if ak else a0.t().contiguous().t()
    b = b0.t().contiguous().t() if bk else b0
    bias = torch.randn(N, generator=g).to(dev)
    c0 = torch.randn(M, N, generator=g).to(dev)
    out = c0.clone()
    k.gemm(a, b, out, bias=bias, alpha=0.5, beta=1.0, fast=True)
    ref = _ref(a0, b0, bias, c0, alpha=0.5, beta=1.0)
    bound = 0.5 * (a0.double().abs() @ b0.double().abs()) * 4e-5 + 1e-5 * (1 + c0.double().abs() + bias.double().abs())
    excess = ((out.double() - ref).abs() - bound).max().item()
    assert excess <= 0, excess
    # and it is not the f32 path in disguise: the error is that of a split-bf16 product (> f32's ~1e-7)
    if M >= 64 and N >= 64 and K >= 64:
        rel = ((out.double() - ref).abs().max() / (a0.double().abs() @ b0.double().abs()).max()).item()
        assert rel > 1e-9, rel


def test_gemm_bf16x3_batched_split():
    from sdreamer import kernels as k
    g = torch.Generator(device="cpu").manual_seed(11)
    a = torch.randn(8, 256, 1024, generator=g).cuda()
    b = torch.randn(8, 1024, 768, generator=g).cuda()
    out = torch.empty(8, 256, 768, device="cuda")
    k.gemm(a, b, out, ksplit=4, fast=True)
    ref = a.double() @ b.double()
    bound = 4e-5 * (a.double().abs() @ b.double().abs()) + 1e-6
    assert ((out.double() - ref).abs() - bound).max().item() <= 0


@pytest.mark.parametrize("M,N,K,n,rms", [(1000, 256, 2560, 4, False), (4096, 256, 256, 2, True),
                                          (2048, 255, 256, 2, True), (300, 128, 96, 1, True),
                                          (12345, 256, 512, 4, False)])
def test_gemm_bf16x3_mlp(M, N, K, n, rms):
    """sd_gemm_bf16x3_mlp: out[b] = silu(rms(x[b]) * nw[b]) @ w[b]^T + bias[b] (RMSNorm from the producer's row
    partials, nn.RMSNorm eps 1e-4) and this layer's row partial sums of squares per 64 columns, against torch fp32
    (split-bf16 tolerance 4e-5 * sum |a||b| per output, as test_gemm_bf16x3_*); x broadcast over the batch when not
    normalised (the imagined heads' first layers; M = 12345 takes the 256 x 256 wide kernel, ragged last row tile)."""
    from sdreamer import kernels as kern
    g = torch.Generator().manual_seed(M + N + K)
    x = torch.randn(n if rms else 1, M, K, generator=g) * 2
    w = torch.randn(n, N, K, generator=g) / K ** 0.5
    b = torch.randn(n, N, generator=g) * 0.1
    nw = 1 + 0.1 * torch.randn(n, K, generator=g)
    if rms:
        a = x / torch.sqrt((x * x).mean(-1, keepdim=True) + 1e-4) * nw[:, None]
        a = a * torch.sigmoid(a)
        pin = torch.stack([(x[:, :, c:c + 64] ** 2).sum(-1) for c in range(0, K, 64)], 1)  # (n, K/64, M)
    else:
        a = x.expand(n, M, K)
    ref = torch.einsum("bmk,bnk->bmn", a.double(), w.double()) + b.double()[:, None]
    bound = torch.einsum("bmk,bnk->bmn", a.abs().double(), w.abs().double()) * 4e-5 + 1e-6
    xd = x.to("cuda") if rms else x.to("cuda").expand(n, M, K)
    out = torch.empty(n, M, N, device="cuda")
    pout = torch.empty(n, N // 64, M, device="cuda") if N % 64 == 0 else None
    ok = kern.mlp_layer(xd, w.to("cuda"), out, bias=b.to("cuda"), norm_w=nw.to("cuda") if rms else None,
                     part_in=pin.to("cuda") if rms else None, part_out=pout)
    assert ok
    err = (out.double().cpu() - ref).abs()
    assert (err <= bound).all(), float((err - bound).max())
    if pout is not None:
        o = out.double().cpu()
        pref = torch.stack([(o[:, :, c:c + 64] ** 2).sum(-1) for c in range(0, N, 64)], 1)
        assert torch.allclose(pout.double().cpu(), pref, rtol=1e-5, atol=1e-6)


def test_heads_fused_match_unfused():
    """networks.heads_nograd's fused path (every layer one batched sd_gemm_bf16x3_mlp launch) against the per-head
    fp32 forwards on the same rows: the four imagined heads of the walker agent (reward / continue 1 hidden layer,
    value / slow value 3)."""
    from sdreamer.networks import heads_nograd
    from test_gpu_dreamer import build_agent
    ag, _, _, _ = build_agent("walker_r2")
    heads = (ag.reward, ag.cont, ag.value, ag._slow_value)
    F = heads[0].mlp._mods[0][0].weight.shape[1]
    x = torch.randn(2048, F, generator=torch.Generator().manual_seed(3)).to("cuda")
    got = heads_nograd(heads, x, True)
    for h, gl in zip(heads, got):
        ref = h.logits_nograd(x, False)
        scale = float(ref.abs().max()) + 1e-6
        assert float((gl - ref).abs().max()) <= 2e-4 * scale, (float((gl - ref).abs().max()), scale)


@pytest.mark.parametrize("R,O,I", [(15360, 256, 2560), (8192, 200, 300), (1024, 255, 256), (4096, 512, 256), (100, 64, 64)])
def test_wgrad_fused_bias(R, O, I):
    """kernels.wgrad: dw += dy^T x on the split-bf16 path with db += column sums of dy fused into the same launch
    (sd_gemm_bf16x3_wgrad, split-K partials summed by the reduce launch) against torch fp32; the column sums to
    1e-5 relative (fp32 sums in a fixed order), dw to the split-bf16 bound."""
    from sdreamer import kernels as kern
    g = torch.Generator().manual_seed(R + O)
    dy = torch.randn(R, O, generator=g)
    x = torch.randn(R, I, generator=g)
    dw0 = torch.randn(O, I, generator=g)
    db0 = torch.randn(O, generator=g)
    dw, db = dw0.clone().to("cuda"), db0.clone().to("cuda")
    kern.wgrad(dy.to("cuda"), x.to("cuda"), dw, db)
    ref = dw0.double() + dy.double().t() @ x.double()
    bound = (dy.abs().double().t() @ x.abs().double()) * 4e-5 + 1e-5
    assert ((dw.double().cpu() - ref).abs() <= bound).all()
    dref = db0.double() + dy.double().sum(0)
    assert torch.allclose(db.double().cpu(), dref, rtol=1e-5, atol=1e-4 * float(dy.abs().sum(0).max()) * 1e-2)


@pytest.mark.parametrize("rms,wide", [(False, False), (True, False), (False, True)])
def test_gemm_bf16x3_mlp_entries(rms, wide):
    """sd_gemm_bf16x3_mlp's per-entry operands (sd_mlp_ext.w_ptr / bias_ptr / norm_w_ptr / w_rows): separate weight
    tensors of different row counts in one launch, bit-identical to the stacked, zero-padded batch (what
    networks._heads_rest_fused did before), columns past an entry's rows exactly 0 (wide: N = 256 over 12,800 rows,
    the 256 x 256 kernel)."""
    from sdreamer import kernels as kern
    g = torch.Generator().manual_seed(7)
    M, K, N = (12800, 256, 256) if wide else (1500, 256, 255)
    rows = [256, 1, 256, 64] if wide else [255, 1, 255, 64]
    n = len(rows)
    x = (torch.randn(n if rms else 1, M, K, generator=g) * 2).cuda()
    ws = [(torch.randn(r, K, generator=g) / 16).cuda() for r in rows]
    bs = [torch.randn(r, generator=g).cuda() for r in rows]
    nws = [(1 + 0.1 * torch.randn(K, generator=g)).cuda() for _ in rows]
    pin = torch.stack([(x[:, :, c:c + 64] ** 2).sum(-1) for c in range(0, K, 64)], 1).contiguous() if rms else None
    xd = x if rms else x.expand(n, M, K)
    wst = torch.zeros(n, N, K, device="cuda")
    bst = torch.zeros(n, N, device="cuda")
    for j, (w, b) in enumerate(zip(ws, bs)):
        wst[j, :w.shape[0]] = w
        bst[j, :w.shape[0]] = b
    ref = torch.empty(n, M, N, device="cuda")
    got = torch.full((n, M, N), float("nan"), device="cuda")
    kw = dict(part_in=pin) if rms else {}
    assert kern.mlp_layer(xd, wst, ref, bias=bst, norm_w=torch.stack(nws) if rms else None, **kw)
    assert kern.mlp_layer(xd, ws, got, bias=bs, norm_w=nws if rms else None, **kw)
    assert torch.equal(got, ref)
    for j, r in enumerate(rows):
        assert not got[j, :, r:].any()


def test_heads_w256_matches_128_tiles():
    """The imagined heads at the bench's row count (H1 * N = 16 * 1024): their first layer takes the 256 x 256-tile
    kernel (gemm3_w256_kernel, 32x32x16 MFMAs: its own k order) — against the same launch on the 128-tile kernel
    (SDHIP_MLP_NOW256) and against the per-head fp32 forwards, every head's logits at the split-bf16 bound."""
    from sdreamer.networks import heads_nograd
    from test_gpu_dreamer import build_agent
    ag, _, _, _ = build_agent("walker_r2")
    heads = (ag.reward, ag.cont, ag.value, ag._slow_value)
    F = heads[0].mlp._mods[0][0].weight.shape[1]
    x = torch.randn(16384, F, generator=torch.Generator().manual_seed(5)).to("cuda")
    f0 = []
    got = heads_nograd(heads, x, True, firsts_out=f0)
    os.environ["SDHIP_MLP_NOW256"] = "1"
    try:
        f1 = []
        alt = heads_nograd(heads, x, True, firsts_out=f1)
    finally:
        del os.environ["SDHIP_MLP_NOW256"]
    s0 = float(f1[0].abs().max())
    assert float((f0[0] - f1[0]).abs().max()) <= 1e-4 * s0  # the first layers: same products, other k order
    assert not torch.equal(f0[0], f1[0])  # (the two kernels did run: their sums differ in rounding)
    for h, g, a in zip(heads, got, alt):
        ref = h.logits_nograd(x, False)
        scale = float(ref.abs().max()) + 1e-6
        assert float((g - ref).abs().max()) <= 2e-4 * scale, (float((g - ref).abs().max()), scale)
        assert float((g - a).abs().max()) <= 2e-4 * scale


@pytest.mark.parametrize("R,O,I", [(15360, 256, 2560), (4096, 128, 512)])
def test_wgrad2_matches_two_wgrads(R, O, I):
    """kernels.wgrad2 (two layers' weight gradients over one input: one GEMM over the joint dy, rows >= split's bias
    gradients into the second buffer) against torch fp32 at the split-bf16 bound, and the bias sums to 1e-5."""
    from sdreamer import kernels as kern
    g = torch.Generator().manual_seed(R + 2 * O)
    dy = torch.randn(R, 2 * O, generator=g)
    x = torch.randn(R, I, generator=g)
    dw0 = torch.randn(2 * O, I, generator=g)
    da0, db0 = torch.randn(O, generator=g), torch.randn(O, generator=g)
    dw, da, db = dw0.clone().to("cuda"), da0.clone().to("cuda"), db0.clone().to("cuda")
    kern.wgrad2(dy.to("cuda"), x.to("cuda"), dw, da, db, O)
    ref = dw0.double() + dy.double().t() @ x.double()
    bound = (dy.abs().double().t() @ x.abs().double()) * 4e-5 + 1e-5
    assert ((dw.double().cpu() - ref).abs() <= bound).all()
    s = dy.double().sum(0)
    tol = 1e-4 * float(dy.abs().sum(0).max()) * 1e-2
    assert torch.allclose(da.double().cpu(), da0.double() + s[:O], rtol=1e-5, atol=tol)
    assert torch.allclose(db.double().cpu(), db0.double() + s[O:], rtol=1e-5, atol=tol)
