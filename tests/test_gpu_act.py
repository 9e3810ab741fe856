"""Dreamer.act (dreamer.py:330-357) on the GPU vs the oracle restatement (oracle/ref_cpu.py Oracle.act), and the
graph-replayed policy (Dreamer.policy_graph, the per-env-step latency path) vs eager act. Stated tolerances: posterior
latent indices bit-exact (no near-tie in these draws), deter / actions <= 1e-4 abs (f32 contractions in a different
order), discrete actions exact; the replayed graph equals eager act bit for bit."""
import numpy as np
import pytest
import torch

from oracle.ref_cpu import Oracle
from test_gpu_dreamer import build_agent

pytestmark = pytest.mark.gpu


def _inputs(spec, obs_shapes, B, A, discrete, seed):
    g = torch.Generator().manual_seed(seed)
    obs = {k: torch.randint(0, 256, (B,) + tuple(v), dtype=torch.uint8, generator=g) for k, v in obs_shapes.items()}
    obs["is_first"] = torch.tensor([i % 3 == 0 for i in range(B)])
    idx = torch.randint(0, spec.K, (B, spec.S), generator=g)
    a = torch.nn.functional.one_hot(torch.randint(0, A, (B,), generator=g), A).float() if discrete else \
        torch.rand(B, A, generator=g) * 2 - 1
    state = {"stoch": torch.nn.functional.one_hot(idx, spec.K).float(), "deter": 0.3 * torch.randn(B, spec.D, generator=g),
             "prev_action": a}
    return obs, state


@pytest.mark.parametrize("name", ["walker_r2", "atari_r2"])
@pytest.mark.parametrize("ev", [False, True])
def test_act_matches_oracle(name, ev):
    ag, z, spec, obs_shapes = build_agent(name)
    A, discrete = int(z["meta_A"]), bool(z["meta_discrete"])
    M = Oracle(spec, {k: torch.from_numpy(v) for k, v in __import__("golden_io").load_case(name)[3].items()})
    obs, state = _inputs(spec, obs_shapes, 6, A, discrete, 5)
    a_ref, s_ref = M.act(obs, state, seed=321, step=4, eval=ev)
    a, s = ag.act({k: v.cuda() for k, v in obs.items()}, {k: v.cuda() for k, v in state.items()}, eval=ev,
                  seed=321, step=4)
    assert torch.equal(s["stoch"].argmax(-1).cpu(), s_ref["stoch"].argmax(-1))
    np.testing.assert_allclose(s["deter"].cpu().numpy(), s_ref["deter"].numpy(), atol=1e-4)
    if discrete:
        assert torch.equal(a.cpu(), a_ref)
    else:
        np.testing.assert_allclose(a.cpu().numpy(), a_ref.numpy(), atol=1e-4)


def test_policy_graph_equals_eager_act():
    ag, z, spec, obs_shapes = build_agent("walker_r2")
    A = int(z["meta_A"])
    obs, state = _inputs(spec, obs_shapes, 8, A, False, 9)
    obs = {k: v.cuda() for k, v in obs.items()}
    state = {k: v.cuda() for k, v in state.items()}
    policy = ag.policy_graph(8, obs)
    base = ag._seed_base + 7
    st_g, st_e = dict(state), dict(state)
    for k in range(3):
        a_g, st_g = policy(obs, st_g)
        a_g, st_g = a_g.clone(), {n: v.clone() for n, v in st_g.items()}
        a_e, st_e = ag.act(obs, st_e, seed=base + k, step=0)
        assert torch.equal(a_g, a_e), k
        for n in st_e:
            assert torch.equal(st_g[n], st_e[n]), (k, n)
        obs["is_first"] = torch.zeros_like(obs["is_first"])


def test_video_pred_decoder_agent():
    """dreamer.py:366-400 on the decoder (rep_loss=dreamer) agent: layout cat([truth, model, error], 2), the first
    5 model frames are the decoded posterior, the rest open-loop; deterministic for a fixed seed."""
    ag, z, spec, obs = build_agent("walker_dreamer")
    g = torch.Generator().manual_seed(4)
    B0, T, A = 3, 9, int(z["meta_A"])
    first = torch.zeros(B0, T, 1, dtype=torch.bool)
    first[:, 0] = True
    data = {"image": torch.randint(0, 256, (B0, T, 64, 64, 3), dtype=torch.uint8, generator=g).cuda(),
            "action": (torch.rand(B0, T, A, generator=g) * 2 - 1).cuda(), "is_first": first.cuda()}
    init = (torch.zeros(B0, spec.S, spec.K, device="cuda"), torch.zeros(B0, spec.D, device="cuda"))
    v1 = ag.video_pred(dict(data), init, seed=3)
    v2 = ag.video_pred(dict(data), init, seed=3)
    B = min(data["action"].shape[0], 6)
    assert tuple(v1.shape) == (B, T, 3 * 64, 64, 3) and torch.isfinite(v1).all()
    assert torch.equal(v1, v2)
    truth = data["image"][:B].float() / 255.0
    assert torch.allclose(v1[:, :, :64], truth)
    model = v1[:, :, 64:128]
    assert torch.allclose(v1[:, :, 128:], (model - truth + 1.0) / 2.0)


def test_video_pred_matches_reference():
    """Dreamer.video_pred vs the reference's own (golden vp_*, tests/golden/gen_golden.py video_case): walker decoder
    agent at the initial weights, B2 T8 — posterior over 5 steps (noise STREAM_OBS step i), open-loop
    imagine_with_action over the last 3 logged actions (STREAM_IMG step i), decoded; subsampled output within 1e-4."""
    ag, z, spec, obs = build_agent("walker_dreamer")
    data = {k: torch.from_numpy(z[f"vp_in_{k}"]).cuda()
            for k in ("image", "action", "reward", "is_first", "is_terminal", "is_last")}
    idx = torch.from_numpy(z["vp_in_init_stoch"].astype(np.int64))
    init = (torch.nn.functional.one_hot(idx, spec.K).float().cuda(), torch.from_numpy(z["vp_in_init_deter"]).cuda())
    vid = ag.video_pred(data, init, seed=int(z["vp_seed"]))
    assert tuple(vid.shape) == tuple(z["vp_shape"])
    got = vid[:, :, ::4, ::4, :].cpu().numpy()
    np.testing.assert_allclose(got, z["vp_out"], rtol=1e-4, atol=1e-4)
