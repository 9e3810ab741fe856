"""GEMM kernel (sd_gemm_f32) vs torch fp32 reference, all operand layouts, batching, split-K, bias/beta."""
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
