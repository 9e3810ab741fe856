"""Fused imagination (csrc/img.hip: 9 launches per step) against the per-op HIP path (pinned end-to-end to the
reference's golden vectors in test_gpu_dreamer.py), with the golden agents' weights: continuous actor (walker),
discrete actor + 32x32 latents (atari), deter 4096 (memory maze); N aligned to the 64-row tiles and ragged.
Tolerances: feats/actions 1e-3 rel + 2e-4 abs (different fp32 summation order); sampled latent indices must agree
except on near-ties (at most 0.1% of the categoricals)."""
import pytest
import torch

from sdreamer import dreamer as DR
from test_gpu_dreamer import build_agent

pytestmark = pytest.mark.gpu


def _start(ag, N, seed):
    g = torch.Generator().manual_seed(seed)
    S, Kd, D = ag.rssm._stoch, ag.rssm._discrete, ag.rssm._deter
    idx = torch.randint(0, Kd, (N, S), generator=g)
    stoch = torch.nn.functional.one_hot(idx, Kd).float().cuda()
    deter = (0.5 * torch.randn(N, D, generator=g)).cuda()
    return stoch, deter


def _run(ag, start, H1, fused):
    DR.FUSED_IMAG = fused
    try:
        f, a = ag._imagine_tm(start, H1, seed=77, row_offset=5)
        torch.cuda.synchronize()
        return f.clone(), a.clone()
    finally:
        DR.FUSED_IMAG = True


@pytest.mark.parametrize("name", ["walker_r2", "atari_r2", "maze_r2"])
@pytest.mark.parametrize("N", [128, 100])
def test_fused_imagination_matches_per_op(name, N):
    ag, z, spec, obs = build_agent(name)
    assert ag._fused_imag_ok()
    start = _start(ag, N, 3)
    H1 = 6
    fr, ar = _run(ag, start, H1, False)
    ff, af = _run(ag, start, H1, True)
    SK = ag.rssm.flat_stoch
    Kd = ag.rssm._discrete
    ir = fr[:, :, :SK].reshape(H1, N, -1, Kd).argmax(-1)
    i_f = ff[:, :, :SK].reshape(H1, N, -1, Kd).argmax(-1)
    mism = (ir != i_f).float().mean().item()
    assert mism <= 1e-3, mism
    if mism == 0:
        torch.testing.assert_close(ff, fr, rtol=1e-3, atol=2e-4)
        torch.testing.assert_close(af, ar, rtol=1e-3, atol=2e-4)
    else:  # compare up to the first step with a flipped sample
        t0 = int((ir != i_f).flatten(1).any(1).nonzero()[0])
        torch.testing.assert_close(ff[:t0 + 1, :, SK:], fr[:t0 + 1, :, SK:], rtol=1e-3, atol=2e-4)
        torch.testing.assert_close(af[:t0 + 1], ar[:t0 + 1], rtol=1e-3, atol=2e-4)


def test_fused_imagination_deterministic():
    ag, z, spec, obs = build_agent("walker_r2")
    start = _start(ag, 192, 5)
    a = _run(ag, start, 5, True)
    b = _run(ag, start, 5, True)
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])


@pytest.mark.parametrize("name,N", [("walker_r2", 192), ("atari_r2", 100), ("maze_r2", 128)])
def test_presplit_images_bit_identical(name, N):
    """k_hid reading deter / x1 / x2 from their producers' pre-split bf16x3 images (KH_APRE; on k_hid_areg also x0,
    from k_action_rows) gives exactly the imagination of the in-loader split (SDHIP_KH_NOAPRE): the same fp32 values
    are split, x0's and x1's rstd are summed in wg_rstd's order."""
    import os
    ag, z, spec, obs = build_agent(name)
    start = _start(ag, N, 11)
    os.environ["SDHIP_KL_NOPRE"] = "1"  # k_lin6 needs the deter image: compare the k_hid paths on the fp32 k_lin
    try:
        a = _run(ag, start, 6, True)
        os.environ["SDHIP_KH_NOAPRE"] = "1"
        b = _run(ag, start, 6, True)
    finally:
        os.environ.pop("SDHIP_KH_NOAPRE", None)
        del os.environ["SDHIP_KL_NOPRE"]
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])


@pytest.mark.parametrize("name,N", [("walker_r2", 96), ("atari_r2", 64)])
def test_lin6_matches_fp32_lin(name, N):
    """The deter contractions on pre-split operands (k_lin6, bf16x6: fp32-accurate) against the fp32 k_lin
    (SDHIP_KL_NOPRE): same imagined indices except near-ties, deter / actions to fp32 rounding."""
    import os
    ag, z, spec, obs = build_agent(name)
    start = _start(ag, N, 13)
    a = _run(ag, start, 6, True)
    os.environ["SDHIP_KL_NOPRE"] = "1"
    try:
        b = _run(ag, start, 6, True)
    finally:
        del os.environ["SDHIP_KL_NOPRE"]
    SK = ag.rssm.flat_stoch
    ia = a[0][..., :SK].reshape(*a[0].shape[:2], -1, ag.rssm._discrete).argmax(-1)
    ib = b[0][..., :SK].reshape(*b[0].shape[:2], -1, ag.rssm._discrete).argmax(-1)
    rows_same = (ia == ib).reshape(ia.shape[0], ia.shape[1], -1).all(-1).all(0)  # rows with no index flip
    assert rows_same.float().mean() >= 0.98
    da, db = a[0][:, rows_same, SK:], b[0][:, rows_same, SK:]
    assert (da - db).abs().max() <= 1e-5 * (1 + db.abs().max())


@pytest.mark.parametrize("name,N", [("walker_r2", 192), ("atari_r2", 100), ("maze_r2", 128)])
def test_lin6_areg_matches_lin6(name, N):
    """k_lin6_areg (the deter contractions as 64-row tiles whose K range is split between two halves of the
    workgroup; D = 2048 and maze's 4096) against k_lin6 (SDHIP_KL_NOAREG): the same bf16x6 products, summed as two
    halves then added — fp32 rounding apart, so the same imagined indices except near-ties and deter / actions within
    1e-5 relative."""
    import os
    ag, z, spec, obs = build_agent(name)
    start = _start(ag, N, 19)
    a = _run(ag, start, 6, True)
    os.environ["SDHIP_KL_NOAREG"] = "1"
    try:
        b = _run(ag, start, 6, True)
    finally:
        del os.environ["SDHIP_KL_NOAREG"]
    assert ag.rssm._deter in (2048, 4096)
    SK = ag.rssm.flat_stoch
    ia = a[0][..., :SK].reshape(*a[0].shape[:2], -1, ag.rssm._discrete).argmax(-1)
    ib = b[0][..., :SK].reshape(*b[0].shape[:2], -1, ag.rssm._discrete).argmax(-1)
    rows_same = (ia == ib).reshape(ia.shape[0], ia.shape[1], -1).all(-1).all(0)
    assert rows_same.float().mean() >= 0.98
    da, db = a[0][:, rows_same, SK:], b[0][:, rows_same, SK:]
    assert (da - db).abs().max() <= 1e-5 * (1 + db.abs().max())
    assert not torch.equal(a[0], b[0]), "k_lin6_areg did not run"


@pytest.mark.parametrize("name,N", [("walker_r2", 192), ("atari_r2", 100), ("maze_r2", 128)])
def test_lin6_areg_tiles_bit_identical(name, N):
    """k_lin6_areg's 48-column tiles over the three problems' concatenated columns (pieces of two problems in one
    tile) against its 64-column tiles (SDHIP_KL_NSUB4): the same k order per element, so the same bits."""
    import os
    ag, z, spec, obs = build_agent(name)
    start = _start(ag, N, 23)
    a = _run(ag, start, 6, True)
    os.environ["SDHIP_KL_NSUB4"] = "1"
    try:
        b = _run(ag, start, 6, True)
    finally:
        del os.environ["SDHIP_KL_NSUB4"]
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])


@pytest.mark.parametrize("name,N", [("walker_r2", 192), ("atari_r2", 100), ("maze_r2", 128)])
def test_hid_areg_bit_identical(name, N):
    """k_hid_areg (register A operands from the pre-split images, one fully unrolled K loop; Dg 256 and 512) gives
    exactly k_hid<true>'s imagination (SDHIP_KH_NOAREG): same planes, same six products per k tile in the same order."""
    import os
    ag, z, spec, obs = build_agent(name)
    start = _start(ag, N, 17)
    a = _run(ag, start, 6, True)
    os.environ["SDHIP_KH_NOAREG"] = "1"
    try:
        b = _run(ag, start, 6, True)
    finally:
        del os.environ["SDHIP_KH_NOAREG"]
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])
