"""The update the bench times, pinned at the benched sizes (VERDICT r03 "next" item 1).

bench.py times `Dreamer.update(buffer)` after its warm-up: from the third update on that is the twelve-phase,
two-stream HIP-graph replay (dreamer.py `_update_graphed`) fed by `Buffer.sample_into` (one gather launch into the
graphs' input buffers). The eager first update is pinned to the reference at full size (test_gpu_fullsize.py); this
file pins the replayed schedule to that eager path bit for bit: two agents with the same initial weights and two
identical synthetic replay buffers (bench.synth_buffer) run 5 updates each through `update(buffer)`, one eager
(`use_graphs = False`, Buffer.sample + update_batch), one as the bench runs it (updates 0-1 eager, 2 captured,
3-4 replayed with sample_into). Every metric of every update, the posterior deter / latent indices, the latents
written back into the replay storage and every parameter after the 5th update must be identical.

Workloads: C2 walker r2dreamer B16 L64 H15 (the bench line), C4 atari-like B32 (two 16-row scan tiles), C5
memory-maze-like B16 L256 H25 deter 4096. Reference: /root/reference/world_model/dreamer.py:402-451.
"""
import pytest
import torch

from bench import WORKLOADS, _Sp, _Spaces, synth_buffer

pytestmark = pytest.mark.gpu

N_UPDATES = 5


def _run(config, graphs):
    from sdreamer.config import load_config
    from sdreamer.dreamer import Dreamer
    A, discrete, _ = WORKLOADS[config]
    cfg = load_config(config, ["device=cuda:0", "model.compile=False"])
    torch.manual_seed(0)
    act = _Sp((A,))
    if discrete:
        act.discrete = True
    ag = Dreamer(cfg.model, _Spaces({"image": _Sp((64, 64, 3))}), act)
    ag.use_graphs = graphs
    L = int(cfg.batch_length)
    buf = synth_buffer(cfg, torch.device("cuda:0"), 0, T=max(160, 2 * (L + 1)), A=A, discrete=discrete)
    out = []
    for _ in range(N_UPDATES):
        mets = ag.update(buf)
        torch.cuda.synchronize()
        vals = {k: float(v) for k, v in mets.items()}
        out.append(vals)
    if graphs:
        assert ag._graph is not None, "the graphed run never captured"
    post = ag._g_post if graphs else None
    sd = ag.state_dict()
    params = {k: v.detach().cpu().clone() for k, v in sd.items() if torch.is_tensor(v)}
    store = {k: buf._store[k].cpu().clone() for k in ("stoch", "deter")}
    del ag, buf
    torch.cuda.empty_cache()
    return out, params, store, post


@pytest.mark.parametrize("config", ["dmc/cnn", "dmc/atari_breakout", "dmc/memory_maze"])
def test_graph_replay_matches_eager_fullsize(config):
    e_mets, e_par, e_store, _ = _run(config, False)
    g_mets, g_par, g_store, _ = _run(config, True)
    for u in range(N_UPDATES):
        assert e_mets[u].keys() == g_mets[u].keys()
        diff = {k: (e_mets[u][k], g_mets[u][k]) for k in e_mets[u]
                if not (e_mets[u][k] == g_mets[u][k] or (e_mets[u][k] != e_mets[u][k] and g_mets[u][k] != g_mets[u][k]))}
        assert not diff, f"update {u}: metrics differ {diff}"
    for k in ("stoch", "deter"):  # every posterior latent written back by the 5 updates (buffer.py:44-53)
        assert torch.equal(e_store[k], g_store[k]), f"replay storage {k} differs"
    assert e_par.keys() == g_par.keys()
    bad = [k for k in e_par if not torch.equal(e_par[k], g_par[k])]
    assert not bad, f"parameters differ after {N_UPDATES} updates: {bad[:8]}"
