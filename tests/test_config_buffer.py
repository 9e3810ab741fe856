"""Config surface (configs/base.yaml key layout, Hydra-style overrides) and replay-buffer semantics
(utils/buffer.py:27-53: B slices of L+1 steps inside one episode, action shifted one step back,
`initial` = stored latent at slice step 0, latent write-back)."""
import torch

from sdreamer.buffer import Buffer
from sdreamer.config import load_config


def test_config_defaults_and_overrides():
    c = load_config("dmc/cnn", ["model.lr=1e-4", "batch_size=8", "+model.new_key=3"])
    assert c.model.lr == 1e-4 and isinstance(c.model.eps, float) and c.model.eps == 1e-20
    assert c.buffer.batch_size == 8 and c.trainer.batch_size == 8  # interpolation follows the override
    assert c.model.rssm.deter == 2048 and c.model.rssm.discrete == 16 and c.model.rssm.stoch == 32
    assert c.model.rep_loss == "r2dreamer" and c.model.imag_horizon == 15 and c.model.horizon == 333
    assert dict(c.model.loss_scales)["barlow"] == 0.05 and c.model.new_key == 3
    assert c.model.encoder.cnn.mults == [2, 3, 4, 4] and c.model.critic.dist.bin_num == 255
    p = load_config("dmc/proprio")
    assert p.model.rep_loss == "dreamer" and p.batch_size == 4 and p.model.encoder.mlp_keys == "(position|velocity)"
    m = load_config("dmc/memory_maze")
    assert m.model.rssm.deter == 4096 and m.batch_length == 256 and m.model.imag_horizon == 25


def _buffer(E=4, T=40, L=8, B=6):
    cfg = load_config("dmc/cnn", ["device=cpu", f"batch_size={B}", f"batch_length={L}", "buffer.storage_device=cpu"])
    buf = Buffer(cfg.buffer, device="cpu", seed=3)
    ep = torch.zeros(T, E, dtype=torch.int32)
    ep[T // 2:] = 1  # an episode boundary in the middle of every env's stream
    data = {"action": torch.arange(T * E, dtype=torch.float32).view(T, E, 1).repeat(1, 1, 2),
            "t": torch.arange(T).view(T, 1).expand(T, E).clone(), "env": torch.arange(E).view(1, E).expand(T, E).clone(),
            "episode": ep, "stoch": torch.randn(T, E, 3, 4), "deter": torch.randn(T, E, 5)}
    for i in range(T):
        buf.add_transition({k: v[i] for k, v in data.items()})
    return buf, data


def test_buffer_sample_semantics():
    buf, src = _buffer()
    L = buf.batch_length
    for _ in range(5):
        data, index, initial = buf.sample()
        t_idx, e_idx = index
        assert data["action"].shape == (buf.batch_size, L, 2)
        t0 = data["t"][:, 0] - 1  # slice start (stored step 0 is not returned as data)
        env = data["env"][:, 0]
        assert torch.equal(data["t"], t0[:, None] + 1 + torch.arange(L)[None])  # consecutive steps
        assert torch.equal(data["env"], env[:, None].expand(-1, L))
        ep = src["episode"][t0, env]
        assert torch.equal(src["episode"][t0 + L, env], ep)  # slice stays inside one episode
        exp_act = src["action"][t0[:, None] + torch.arange(L)[None], env[:, None]]
        assert torch.equal(data["action"], exp_act)  # action one step back
        assert torch.equal(initial[0], src["stoch"][t0, env]) and torch.equal(initial[1], src["deter"][t0, env])
        assert torch.equal(t_idx, t0[:, None] + 1 + torch.arange(L)[None])


def test_buffer_update_writes_back():
    buf, src = _buffer()
    data, index, initial = buf.sample()
    st = torch.full((buf.batch_size, buf.batch_length, 3, 4), 7.0)
    de = torch.full((buf.batch_size, buf.batch_length, 5), -2.0)
    buf.update(index, st, de)
    t_idx, e_idx = index
    assert torch.all(buf._store["stoch"][t_idx, e_idx] == 7.0)
    assert torch.all(buf._store["deter"][t_idx, e_idx] == -2.0)
    assert buf.count() == 40 * 4


def test_buffer_update_overlapping_slices_last_row_wins():
    """Overlapping slices write one storage row several times; the slice with the largest b wins (deterministic,
    the rule sd_replay_slices' scatter follows)."""
    buf, src = _buffer()
    L = buf.batch_length
    # slices 0 and 2 overlap on env 1 (starts 3 and 5), slice 1 on env 2 is disjoint, slice 3 repeats slice 0
    t0 = torch.tensor([3, 10, 5, 3])
    env = torch.tensor([1, 2, 1, 1])
    B = len(t0)
    t_idx = (t0[:, None] + 1 + torch.arange(L)[None]) % buf.cap
    e_idx = env[:, None].expand(B, L)
    st = torch.arange(B, dtype=torch.float32).reshape(B, 1, 1, 1).expand(B, L, 3, 4).contiguous()
    de = torch.arange(B, dtype=torch.float32).reshape(B, 1, 1).expand(B, L, 5).contiguous()
    buf.update([t_idx, e_idx], st, de)
    for b in range(B):
        for j in range(L):
            t, e = int(t_idx[b, j]), int(env[b])
            writers = [b2 for b2 in range(B) if int(env[b2]) == e and t in t_idx[b2].tolist()]
            assert float(buf._store["deter"][t, e, 0]) == max(writers)
            assert float(buf._store["stoch"][t, e, 0, 0]) == max(writers)
