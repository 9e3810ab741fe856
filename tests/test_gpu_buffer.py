"""Fused replay slices (sd_replay_slices): Buffer.sample_into / the fused write-back equal sample() / update()
bit for bit (same generator stream -> same slices), including the one-step action shift and the initial latents."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _buffer(seed):
    from sdreamer.buffer import Buffer
    from sdreamer.config import load_config
    cfg = load_config("dmc/cnn", ["device=cuda:0", "batch_size=4", "batch_length=6"])
    g = torch.Generator().manual_seed(3)
    T, E = 40, 3
    buf = Buffer(cfg.buffer, device="cuda:0", seed=seed)
    ep = torch.zeros(T, E, dtype=torch.int32)
    ep[20:] = 1  # an episode boundary: slices must not cross it
    buf.add_sequence({
        "image": torch.randint(0, 256, (T, E, 8, 8, 3), dtype=torch.uint8, generator=g).cuda(),
        "action": torch.randn(T, E, 6, generator=g).cuda(),
        "reward": torch.randn(T, E, 1, generator=g).cuda(),
        "is_first": (torch.rand(T, E, 1, generator=g) < 0.1).cuda(),
        "episode": ep.cuda(),
        "stoch": torch.randn(T, E, 4, 5, generator=g).cuda(),
        "deter": torch.randn(T, E, 7, generator=g).cuda(),
    })
    return buf


def test_sample_into_and_writeback_match_reference_semantics():
    a, b = _buffer(11), _buffer(11)
    for it in range(3):
        data, index, initial = a.sample()
        dst = {k: torch.empty_like(v) for k, v in data.items()}
        dst_init = tuple(torch.empty_like(t) for t in initial)
        idx_b = b.sample_into(dst, dst_init)
        for k in data:
            assert torch.equal(dst[k], data[k]), (it, k)
        assert torch.equal(dst_init[0], initial[0]) and torch.equal(dst_init[1], initial[1])
        assert torch.equal(idx_b[0], index[0]) and torch.equal(idx_b[1], index[1])
        # overlapping slices write the same (t, e) twice: both paths keep the slice with the largest b (values that
        # differ per slice row, so a wrong winner shows)
        B, L = index[0].shape
        key = (torch.arange(B, device=index[0].device)[:, None] * 1000 + torch.arange(L, device=index[0].device)[None]
               + 100 * it).float()
        post_s = key[..., None, None].expand(*index[0].shape, 4, 5).contiguous()
        post_d = key[..., None].expand(*index[0].shape, 7).contiguous() * 0.5
        a.update(index, post_s, post_d)
        b.update(idx_b, post_s, post_d)
        torch.cuda.synchronize()
        for k in a._store:
            assert torch.equal(a._store[k], b._store[k]), (it, k)
