"""Fused RSSM posterior scan (csrc/scan.hip: 4 launches/step forward, 5 backward) against the per-op HIP kernels
(the path that is pinned to the reference's golden vectors in test_gpu_dreamer.py), on the RSSM shapes of the
BASELINE configs: deter 2048 / discrete 16 (dmc), discrete 32 (atari), deter 4096 (memory maze).
Tolerances: forward states / logits 1e-4 abs + 1e-3 rel (different fp32 summation order); sampled one-hot
indices exact unless the perturbed-logit margin is a near-tie; gradients 2e-3 relative to each tensor's max."""
import copy

import pytest
import torch

from sdreamer import rssm as R
from sdreamer.config import load_config

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _model(cfg_name, B, T, E=96, A=6, seed=0):
    cfg = load_config(cfg_name, ["device=cuda:0"])
    m = R.RSSM(copy.deepcopy(cfg.model.rssm), E, A).to(DEV)
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for name, p in m.named_parameters():
            if p.dim() == 1:
                v = 1.0 + 0.1 * torch.randn(p.shape, generator=g) if "norm" in name or "_n_" in name or \
                    name.endswith(("1.weight",)) else 0.1 * torch.randn(p.shape, generator=g)
            else:
                v = torch.randn(p.shape, generator=g) / p.shape[-1] ** 0.5
            p.copy_(v)
    embed = torch.randn(B, T, E, generator=g).to(DEV)
    action = torch.randn(B, T, A, generator=g).to(DEV)
    reset = torch.rand(B, T, generator=g) < 0.15
    reset[:, 0] = True
    S, K, D = m._stoch, m._discrete, m._deter
    init = (torch.zeros(B, S, K, device=DEV), torch.zeros(B, D, device=DEV))
    ups = (torch.randn(B, T, S, K, generator=g).to(DEV), torch.randn(B, T, D, generator=g).to(DEV) * 0.1,
           torch.randn(B, T, S, K, generator=g).to(DEV) * 0.1)
    return m, embed, action, reset.to(DEV), init, ups


def _run(m, embed, action, reset, init, ups, fused):
    R.FUSED_SCAN = fused
    try:
        for p in m.parameters():
            p.grad = torch.zeros_like(p)
        e = embed.clone().requires_grad_(True)
        st, de, lo = m.observe(e, action, init, reset, seed=1234, row_offset=0)
        loss = (st * ups[0]).sum() + (de * ups[1]).sum() + (lo * ups[2]).sum()
        loss.backward()
        torch.cuda.synchronize()
        grads = {n: p.grad.detach().clone() for n, p in m.named_parameters()}
        return st.detach(), de.detach(), lo.detach(), e.grad.detach().clone(), grads
    finally:
        R.FUSED_SCAN = True


@pytest.mark.parametrize("cfg_name,B,T", [("dmc/cnn", 16, 8), ("dmc/cnn", 3, 5), ("dmc/atari_breakout", 16, 6),
                                          ("dmc/memory_maze", 8, 4),
                                          ("dmc/atari_breakout", 32, 5), ("dmc/cnn", 20, 4)])  # > 16 rows: row tiles
def test_fused_scan_matches_per_op(cfg_name, B, T):
    m, embed, action, reset, init, ups = _model(cfg_name, B, T)
    assert R._fused_scan_ok(m, B)  # B > 16 runs as 16-row tiles side by side in every launch
    ref = _run(m, embed, action, reset, init, ups, fused=False)
    got = _run(m, embed, action, reset, init, ups, fused=True)
    assert torch.equal(got[0].argmax(-1), ref[0].argmax(-1)), "posterior samples differ"
    torch.testing.assert_close(got[1], ref[1], rtol=1e-3, atol=1e-4)
    torch.testing.assert_close(got[2], ref[2], rtol=1e-3, atol=1e-4)
    torch.testing.assert_close(got[0], ref[0], rtol=1e-3, atol=1e-4)
    scale = ref[3].abs().max().item()
    assert (got[3] - ref[3]).abs().max().item() <= 2e-3 * scale
    bad = []
    for n, g in ref[4].items():
        s = g.abs().max().item()
        err = (got[4][n] - g).abs().max().item()
        if err > 2e-3 * s + 1e-7:
            bad.append((n, err, s))
    assert not bad, bad


def test_fused_scan_graph_replay_deterministic():
    """Two identical calls give bit-identical results (no atomics, fixed reduction orders)."""
    m, embed, action, reset, init, ups = _model("dmc/cnn", 16, 6, seed=3)
    a = _run(m, embed, action, reset, init, ups, fused=True)
    b = _run(m, embed, action, reset, init, ups, fused=True)
    for x, y in zip(a[:4], b[:4]):
        assert torch.equal(x, y)
    for n in a[4]:
        assert torch.equal(a[4][n], b[4][n]), n


@pytest.mark.parametrize("cfg_name,B,T", [("dmc/cnn", 20, 5), ("dmc/atari_breakout", 32, 4), ("dmc/cnn", 16, 4)])
def test_scan_row_tiles_bit_identical(cfg_name, B, T):
    """The row tile (rows per workgroup, grid z) only changes which workgroup computes a row: every row's products,
    k order and norms are the same, so outputs and gradients are bit-identical for tiles 16, 8 and 5 (a partial
    last tile included)."""
    m, embed, action, reset, init, ups = _model(cfg_name, B, T, seed=7)
    runs = []
    old = R.SCAN_ROW_TILE
    try:
        for rt in (0, 8, 5):
            R.SCAN_ROW_TILE = rt
            runs.append(_run(m, embed, action, reset, init, ups, fused=True))
    finally:
        R.SCAN_ROW_TILE = old
    a = runs[0]
    for b in runs[1:]:
        for x, y in zip(a[:4], b[:4]):
            assert torch.equal(x, y)
        for n in a[4]:
            assert torch.equal(a[4][n], b[4][n]), n


def test_extra_grads_fallback_matches_views():
    """The backward's second posterior-gradient summands (RSSM._bwd_extra, Dreamer._ph_scan_bwd's feat gradient): as
    the two column halves of one (B, T, SK + D) buffer (the benched DxSink path, read in place) and as two separate
    tensors (a non-conforming pair, copied into one buffer by the fallback) — the same sums in the same kernels, so
    bit-identical gradients."""
    B, T = 16, 6
    m, embed, action, reset, init, ups = _model("dmc/cnn", B, T)
    SK, D = m.flat_stoch, m._deter
    g = torch.Generator().manual_seed(7)
    gfeat = (torch.randn(B, T, SK + D, generator=g) * 0.05).to(DEV)
    outs = []
    for extra in ((gfeat[..., :SK], gfeat[..., SK:]),
                  (gfeat[..., :SK].contiguous(), gfeat[..., SK:].contiguous())):
        assert m.takes_extra_grads(B)
        for p in m.parameters():
            p.grad = torch.zeros_like(p)
        e = embed.clone().requires_grad_(True)
        st, de, lo = m.observe(e, action, init, reset, seed=1234, row_offset=0)
        m._bwd_extra = extra
        loss = (st * ups[0]).sum() + (de * ups[1]).sum() + (lo * ups[2]).sum()
        loss.backward()
        torch.cuda.synchronize()
        assert m._bwd_extra is None
        outs.append((e.grad.clone(), {n: p.grad.clone() for n, p in m.named_parameters()}))
    (e0, g0), (e1, g1) = outs
    assert torch.equal(e0, e1)
    for n in g0:
        assert torch.equal(g0[n], g1[n]), n
