"""Generate golden vectors by running the REAL reference (/root/reference) on CPU in the survey container.

Run:  python tests/golden/gen_golden.py     (writes tests/golden/<case>.npz; needs /root/reference)
      python tests/golden/gen_golden.py full [C2_walker_r2 ...]   (full-size fixtures, see full_case)

For each case the reference `Dreamer` (world_model/dreamer.py:22) is built from our config surface
(which mirrors configs/base.yaml key for key), given deterministic weights (oracle/init.py), fed a seeded
synthetic batch through a stub replay buffer, and its own `update()` (dreamer.py:402-451) is run with:
  * autocast replaced by a null context (dreamer.py:420 would enter CPU fp16 autocast — SURVEY §6/§8(c));
  * sampling noise injected: F.gumbel_softmax (distributions.py:33) and Normal.rsample (bounded_normal)
    draw from oracle/noise.py in the exact call order of _cal_grad (observe ×T, prior ×1 (discarded),
    then per imagination step: actor, img_step).
Hooks record encoder/observe/prior/_imagine/_lambda_return outputs. Gradients are recorded as per-tensor
L2 norms + 32 sampled elements; parameters after the LaProp step the same way. Two updates are run per case
so LaProp's lr-EMA state and ReturnEMA carry over.
"""
import contextlib
import json
import os
import sys
import zlib

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "safe-dreamer_amd"))

sys.path.insert(0, os.path.dirname(HERE))
from fullsize_io import FULL, full_inputs, fixture_path  # noqa: E402
from fullsize_io import OVERRIDES as FULL_OVR, PARAM_SEED as FULL_PARAM_SEED, ROW_STRIDE as FULL_STRIDE  # noqa: E402
from fullsize_io import SEED as FULL_SEED, sample_idx as full_sample_idx  # noqa: E402
from refimport import import_reference  # noqa: E402

from oracle import noise as nz  # noqa: E402
from oracle.init import params_for  # noqa: E402
from oracle.ref_cpu import Spec  # noqa: E402
from sdreamer.config import load_config  # noqa: E402

CASES = {
    # name: (config, overrides, obs shapes, act_dim, discrete, B, T, H)
    "proprio_dreamer": ("dmc/proprio", [], {"position": (3,), "velocity": (2,)}, 1, False, 4, 16, 8),
    "walker_r2": ("dmc/cnn", [], {"image": (64, 64, 3)}, 6, False, 2, 6, 4),
    # no LR warm-up: the first LaProp step is lr = 4e-5 per element (not 4e-8), so parameter deltas are resolvable
    "walker_r2_nowarm": ("dmc/cnn", ["model.warmup=0"], {"image": (64, 64, 3)}, 6, False, 2, 6, 4),
    "walker_infonce": ("dmc/cnn", ["model.rep_loss=infonce"], {"image": (64, 64, 3)}, 6, False, 2, 6, 4),
    "walker_r2aug": ("dmc/cnn", ["model.r2dreamer.aug.enabled=True"], {"image": (64, 64, 3)}, 6, False, 2, 6, 4),
    "walker_pro": ("dmc/cnn", ["model.rep_loss=dreamerpro"], {"image": (64, 64, 3)}, 6, False, 2, 6, 4),
    "walker_dreamer": ("dmc/walker_dreamer", [], {"image": (64, 64, 3)}, 6, False, 2, 4, 3),
    "atari_r2": ("dmc/atari_breakout", [], {"image": (64, 64, 3)}, 4, True, 2, 4, 3),
    "maze_r2": ("dmc/memory_maze", [], {"image": (64, 64, 3)}, 6, True, 2, 4, 3),
}
PARAM_SEED = 0
N_SAMPLE = 32


def sample_idx(name, numel):
    rng = np.random.default_rng([7, zlib.crc32(name.encode())])
    return np.sort(rng.choice(numel, size=min(N_SAMPLE, numel), replace=False))


def make_batch(rng, obs, A, discrete, B, T):
    data = {}
    for k, shp in obs.items():
        if len(shp) == 3:
            data[k] = rng.integers(0, 256, size=(B, T) + shp, dtype=np.uint8)
        else:
            data[k] = rng.standard_normal((B, T) + shp).astype(np.float32)
    if discrete:
        a = rng.integers(0, A, size=(B, T))
        data["action"] = np.eye(A, dtype=np.float32)[a]
    else:
        data["action"] = rng.uniform(-1.5, 1.5, size=(B, T, A)).astype(np.float32)  # >1 exercises the clip
    data["reward"] = rng.uniform(-2, 3, size=(B, T, 1)).astype(np.float32)
    first = rng.random((B, T, 1)) < 0.1
    first[:, 0] = True
    data["is_first"] = first
    term = rng.random((B, T, 1)) < 0.1
    data["is_terminal"] = term
    data["is_last"] = term | (rng.random((B, T, 1)) < 0.05)
    return data


def make_initial(rng, S, K, D, B):
    idx = rng.integers(0, K, size=(B, S))
    stoch = np.eye(K, dtype=np.float32)[idx]
    deter = (0.5 * rng.standard_normal((B, D))).astype(np.float32)
    return stoch, deter


class NoiseSeq:
    """Injects oracle noise in _cal_grad call order (see module doc)."""

    def __init__(self, T, H1, seed, pro=False):
        self.T, self.H1, self.seed = T, H1, seed
        self.pro = pro  # DreamerPro: a second posterior scan over the augmented 2B batch follows the prior
        self.g = 0
        self.n = 0

    def gumbel(self, shape):
        i = self.g
        self.g += 1
        T = self.T
        if i < T:  # observe step i, (B, S, K)
            B = shape[0]
            return nz.gumbel_block(self.seed, nz.STREAM_OBS, i, B, 0, int(np.prod(shape[1:]))).reshape(shape)
        if i == T:  # prior over (B, T, S, K): sample discarded
            return np.zeros(shape, np.float32)
        if self.pro and i <= 2 * T:  # augmented observe step i - T - 1, (2B, S, K)
            return nz.gumbel_block(self.seed, nz.STREAM_OBS_AUG, i - T - 1, shape[0], 0,
                                   int(np.prod(shape[1:]))).reshape(shape)
        j = i - T - 1 - (T if self.pro else 0)
        N = shape[0]
        if self.discrete_act:
            t, which = divmod(j, 2)
            stream = nz.STREAM_ACT if which == 0 else nz.STREAM_IMG
        else:
            t, stream = j, nz.STREAM_IMG
        return nz.gumbel_block(self.seed, stream, t, N, 0, int(np.prod(shape[1:]))).reshape(shape)

    def normal(self, shape):
        t = self.n
        self.n += 1
        N = shape[0]
        return nz.normal_block(self.seed, nz.STREAM_ACT, t, N, 0, int(np.prod(shape[1:]))).reshape(shape)


def aug_randint(aug, seed, B, T):
    """torch.randint stand-in for random_translate's shifts (dreamer.py:864-868): oracle/noise.aug_shifts."""
    orig = torch.randint

    def randint(low, high=None, size=None, **kw):
        if size is None or size[-1] != 2:
            return orig(low, high, size, **kw)
        sh = nz.aug_shifts(seed, B, 0, T, int(aug.max_delta), bool(aug.same_across_time))  # (B, T, 2): (x, y)
        sh = sh[:, :1] if bool(aug.same_across_time) else sh
        return torch.from_numpy(sh.astype(np.float32)).reshape(size).to(kw.get("dtype") or torch.float32)

    return randint


def patch_randint(cfg, seed, B, T):
    if cfg.model.rep_loss == "dreamerpro":  # augment_data's doubled batch (dreamer.py:731-743)
        torch.randint = aug_randint(cfg.model.dreamer_pro.aug, seed, 2 * B, T)
    elif bool(cfg.model.r2dreamer.aug.enabled):
        torch.randint = aug_randint(cfg.model.r2dreamer.aug, seed, B, T)


def run_case(name, mods, TD):
    cfg_name, ovr, obs, A, discrete, B, T, H = CASES[name]
    cfg = load_config(cfg_name, ["device=cpu", "model.compile=False", f"model.imag_horizon={H}"] + ovr)
    D = mods["world_model.dreamer"]

    class Sp:
        def __init__(s, shape):
            s.shape = shape

    class Spaces:
        def __init__(s, d):
            s.spaces = d

    act_space = Sp((A,))
    if discrete:
        act_space.discrete = True
    torch.manual_seed(0)
    import copy
    ag = D.Dreamer(copy.deepcopy(cfg.model), Spaces({k: Sp(v) for k, v in obs.items()}), act_space)
    spec = Spec(cfg.model, obs, A, discrete)
    sd = ag.state_dict()
    ref_train = [k for k in sd if not k.startswith(("_frozen", "_slow_value", "_ema_"))
                 and k != "return_ema.ema_vals"]
    assert sorted(ref_train) == sorted(spec.shapes), (set(ref_train) ^ set(spec.shapes))
    for k, v in spec.shapes.items():
        assert tuple(sd[k].shape) == tuple(v), (k, sd[k].shape, v)
    init_stats = {}
    for k in spec.shapes:  # the reference's own initialiser (tools.weight_init_ + outscale) under manual_seed(0)
        w = sd[k].detach().double().reshape(-1)
        init_stats[f"init_{k}__stat"] = np.array([w.mean().item(), w.std().item() if w.numel() > 1 else 0.0,
                                                  w.abs().max().item(), float(w.numel())])
    vals = params_for(spec.shapes, PARAM_SEED)
    with torch.no_grad():
        named = dict(ag.named_parameters())
        for k, v in vals.items():
            named[k].data.copy_(torch.from_numpy(v))
        for k, v in named.items():
            if k.startswith("_slow_value."):
                v.data.copy_(torch.from_numpy(vals["value." + k[len("_slow_value."):]]))
    out = {"meta_B": B, "meta_T": T, "meta_H": H, "meta_A": A, "meta_discrete": int(discrete),
           "meta_param_seed": PARAM_SEED}
    out.update(init_stats)

    rng = np.random.default_rng(zlib.crc32(name.encode()))
    D.autocast = lambda **k: contextlib.nullcontext()
    orig_gs = torch.nn.functional.gumbel_softmax
    orig_rs = torch.distributions.Normal.rsample
    rec = {}

    def hook(obj, attr, key, many=False):
        orig = getattr(obj, attr)

        def w(*a, **k):
            r = orig(*a, **k)
            if many:
                rec.setdefault(key, []).append(r)
            else:
                rec.setdefault(key, r)  # first call (DreamerPro's augmented observe comes second)
            return r

        setattr(obj, attr, w)

    hook(ag.rssm, "observe", "observe")
    hook(ag.rssm, "prior", "prior")
    hook(ag, "_imagine", "imagine")
    hook(ag, "_lambda_return", "lret", many=True)
    def enc_hook(m, i, o):  # the first call only, not the aug view; returning None keeps the output
        rec.setdefault("embed", o)

    ag.encoder.register_forward_hook(enc_hook)

    for u in range(2):
        seed = 1000 + u
        data_np = make_batch(rng, obs, A, discrete, B, T)
        init_np = make_initial(rng, spec.S, spec.K, spec.D, B)
        for k, v in data_np.items():
            out[f"u{u}_in_{k}"] = v
        out[f"u{u}_in_init_stoch"] = init_np[0].argmax(-1).astype(np.int16)
        out[f"u{u}_in_init_deter"] = init_np[1]
        out[f"u{u}_seed"] = seed
        seq = NoiseSeq(T, H + 1, seed, cfg.model.rep_loss == "dreamerpro")
        seq.discrete_act = discrete

        def gs(logits, tau=1, hard=False, eps=1e-10, dim=-1):
            g = torch.from_numpy(seq.gumbel(tuple(logits.shape)))
            y_soft = ((logits + g) / tau).softmax(dim)
            index = y_soft.max(dim, keepdim=True)[1]
            y_hard = torch.zeros_like(logits).scatter_(dim, index, 1.0)
            return y_hard - y_soft.detach() + y_soft

        def rs(self, sample_shape=torch.Size()):
            shape = self._extended_shape(sample_shape)
            eps = torch.from_numpy(seq.normal(tuple(shape)))
            return self.loc + eps * self.scale

        torch.nn.functional.gumbel_softmax = gs
        torch.distributions.Normal.rsample = rs
        orig_randint = torch.randint
        patch_randint(cfg, seed, B, T)

        class Buf:
            def sample(self_):
                d = TD({k: torch.from_numpy(v) for k, v in data_np.items()}, batch_size=(B, T))
                return d, None, (torch.from_numpy(init_np[0]), torch.from_numpy(init_np[1]))

            def update(self_, index, stoch, deter):
                rec["wb"] = (stoch, deter)

        rec.clear()
        try:
            mets = ag.update(Buf())
        finally:
            torch.nn.functional.gumbel_softmax = orig_gs
            torch.distributions.Normal.rsample = orig_rs
            torch.randint = orig_randint
        assert seq.g == T + 1 + (T if seq.pro else 0) + (H + 1) * (2 if discrete else 1), seq.g
        assert seq.n == (0 if discrete else H + 1), seq.n
        ps, pdet, plog = rec["observe"]
        out[f"u{u}_post_idx"] = ps.argmax(-1).numpy().astype(np.int16)
        out[f"u{u}_post_deter"] = pdet.detach().numpy()[..., ::4].copy()
        out[f"u{u}_post_logit"] = plog.detach().numpy()
        out[f"u{u}_prior_logit"] = rec["prior"][1].detach().numpy()
        out[f"u{u}_embed"] = rec["embed"].detach().numpy()[..., ::8].copy()
        ifeat, iact = rec["imagine"]
        SK = spec.SK
        out[f"u{u}_imag_idx"] = ifeat[..., :SK].reshape(*ifeat.shape[:2], spec.S, spec.K).argmax(-1).numpy().astype(np.int16)
        out[f"u{u}_imag_deter"] = ifeat[..., SK::16].numpy().copy()
        out[f"u{u}_imag_action"] = iact.numpy()
        out[f"u{u}_imag_ret"] = rec["lret"][0].numpy()
        out[f"u{u}_replay_ret"] = rec["lret"][1].numpy()
        for k, v in mets.items():
            out[f"u{u}_m_{k}"] = np.asarray(float(v), np.float64)
        out[f"u{u}_ema_vals"] = ag.return_ema.ema_vals.numpy().copy()
        named = dict(ag.named_parameters())
        for k in spec.shapes:
            p = named[k]
            flat = p.detach().reshape(-1).numpy()
            idx = sample_idx(k, flat.size)
            out[f"u{u}_p_{k}__n"] = np.asarray(np.linalg.norm(flat.astype(np.float64)))
            out[f"u{u}_p_{k}__s"] = flat[idx]
        st = ag._optimizer.state[named["rssm._img_net.img_net_logit.bias"]]
        out[f"u{u}_laprop_lr1"] = np.asarray(st["exp_avg_lr_1"])
        out[f"u{u}_laprop_lr2"] = np.asarray(st["exp_avg_lr_2"])
        for k in spec.shapes:  # LaProp moments per parameter (laprop.py:62-70), same sampled elements
            stk = ag._optimizer.state[named[k]]
            idx = sample_idx(k, named[k].numel())
            out[f"u{u}_st_{k}__m"] = stk["exp_avg"].reshape(-1).numpy()[idx]
            out[f"u{u}_st_{k}__v"] = stk["exp_avg_sq"].reshape(-1).numpy()[idx]
        for k in spec.slow_names.values():
            flat = named[k].detach().reshape(-1).numpy()
            idx = sample_idx(k, flat.size)
            out[f"u{u}_p_{k}__s"] = flat[idx]
    # grads of the FIRST update are not observable after update(); re-run _cal_grad on update-0 inputs with
    # the initial weights for a gradient fixture.
    layout = optim_layout(ag, mods)
    return out, layout


def optim_layout(ag, mods):
    """What train.py:126-130 would write as optims_state_dict (tools.recursively_collect_optim_state_dict,
    tools.py:298-318): its keys, each optimizer state_dict's structure, and the parameter name behind state index i
    (LaProp's param_groups[0]['params'] follow Dreamer._named_params, dreamer.py:196-227)."""
    osd = mods["utils.tools"].recursively_collect_optim_state_dict(ag)
    names = list(ag._named_params.keys())
    lay = {"optims_keys": list(osd.keys()), "named_params": names, "optimizers": {}}
    for key, sd in osd.items():
        g = sd["param_groups"][0]
        lay["optimizers"][key] = {
            "top_keys": sorted(sd.keys()),
            "n_groups": len(sd["param_groups"]),
            "group": {k: (list(v) if isinstance(v, tuple) else v) for k, v in g.items() if k != "params"},
            "params": list(g["params"]),
            "state_keys": sorted(next(iter(sd["state"].values())).keys()) if sd["state"] else [],
            "n_state": len(sd["state"]),
        }
    return lay


def video_case(name, mods, TD):
    """Dreamer.video_pred (dreamer.py:366-400) at the initial weights on a T=8 batch: posterior over 5 steps (noise
    STREAM_OBS step i), then imagine_with_action over the last 3 logged actions (rssm.py:197-209; noise STREAM_IMG
    step i). Output (B, T, 3*64, 64, 3), stored subsampled [..., ::4, ::4, :]."""
    cfg_name, ovr, obs, A, discrete, _, _, H = CASES[name]
    B, T, seed = 2, 8, 3000
    cfg = load_config(cfg_name, ["device=cpu", "model.compile=False", f"model.imag_horizon={H}"] + ovr)
    D = mods["world_model.dreamer"]
    import copy

    class Sp:
        def __init__(s, shape):
            s.shape = shape

    class Spaces:
        def __init__(s, d):
            s.spaces = d

    ag = D.Dreamer(copy.deepcopy(cfg.model), Spaces({k: Sp(v) for k, v in obs.items()}), Sp((A,)))
    spec = Spec(cfg.model, obs, A, discrete)
    vals = params_for(spec.shapes, PARAM_SEED)
    with torch.no_grad():
        named = dict(ag.named_parameters())
        for k, v in vals.items():
            named[k].data.copy_(torch.from_numpy(v))
    rng = np.random.default_rng(zlib.crc32((name + "/video").encode()))
    data_np = make_batch(rng, obs, A, discrete, B, T)
    init_np = make_initial(rng, spec.S, spec.K, spec.D, B)
    calls = [0]

    def gs(logits, tau=1, hard=False, eps=1e-10, dim=-1):
        i = calls[0]
        calls[0] += 1
        stream, step = (nz.STREAM_OBS, i) if i < 5 else (nz.STREAM_IMG, i - 5)
        g = torch.from_numpy(nz.gumbel_block(seed, stream, step, logits.shape[0], 0,
                                             int(np.prod(logits.shape[1:]))).reshape(logits.shape))
        y_soft = ((logits + g) / tau).softmax(dim)
        index = y_soft.max(dim, keepdim=True)[1]
        return torch.zeros_like(logits).scatter_(dim, index, 1.0) - y_soft.detach() + y_soft

    orig_gs = torch.nn.functional.gumbel_softmax
    torch.nn.functional.gumbel_softmax = gs
    try:
        d = TD({k: torch.from_numpy(v) for k, v in data_np.items()}, batch_size=(B, T))
        vid = ag.video_pred(d, (torch.from_numpy(init_np[0]), torch.from_numpy(init_np[1])))
    finally:
        torch.nn.functional.gumbel_softmax = orig_gs
    assert calls[0] == T, calls[0]
    out = {f"vp_in_{k}": v for k, v in data_np.items()}
    out["vp_in_init_stoch"] = init_np[0].argmax(-1).astype(np.int16)
    out["vp_in_init_deter"] = init_np[1]
    out["vp_seed"] = seed
    out["vp_out"] = vid.numpy()[:, :, ::4, ::4, :].copy()
    out["vp_shape"] = np.asarray(vid.shape)
    return out


def grad_case(name, mods, TD):
    """Gradients (post-backward, pre-AGC) of _cal_grad on update-0 inputs at the initial weights."""
    cfg_name, ovr, obs, A, discrete, B, T, H = CASES[name]
    cfg = load_config(cfg_name, ["device=cpu", "model.compile=False", f"model.imag_horizon={H}"] + ovr)
    D = mods["world_model.dreamer"]
    import copy

    class Sp:
        def __init__(s, shape):
            s.shape = shape

    class Spaces:
        def __init__(s, d):
            s.spaces = d

    act_space = Sp((A,))
    if discrete:
        act_space.discrete = True
    ag = D.Dreamer(copy.deepcopy(cfg.model), Spaces({k: Sp(v) for k, v in obs.items()}), act_space)
    spec = Spec(cfg.model, obs, A, discrete)
    vals = params_for(spec.shapes, PARAM_SEED)
    with torch.no_grad():
        named = dict(ag.named_parameters())
        for k, v in vals.items():
            named[k].data.copy_(torch.from_numpy(v))
        for k, v in named.items():
            if k.startswith("_slow_value."):
                v.data.copy_(torch.from_numpy(vals["value." + k[len("_slow_value."):]]))
    rng = np.random.default_rng(zlib.crc32(name.encode()))
    data_np = make_batch(rng, obs, A, discrete, B, T)
    init_np = make_initial(rng, spec.S, spec.K, spec.D, B)
    seq = NoiseSeq(T, H + 1, 1000, cfg.model.rep_loss == "dreamerpro")
    seq.discrete_act = discrete
    orig_gs = torch.nn.functional.gumbel_softmax
    orig_rs = torch.distributions.Normal.rsample

    def gs(logits, tau=1, hard=False, eps=1e-10, dim=-1):
        g = torch.from_numpy(seq.gumbel(tuple(logits.shape)))
        y_soft = ((logits + g) / tau).softmax(dim)
        index = y_soft.max(dim, keepdim=True)[1]
        y_hard = torch.zeros_like(logits).scatter_(dim, index, 1.0)
        return y_hard - y_soft.detach() + y_soft

    def rs(self, sample_shape=torch.Size()):
        shape = self._extended_shape(sample_shape)
        return self.loc + torch.from_numpy(seq.normal(tuple(shape))) * self.scale

    torch.nn.functional.gumbel_softmax = gs
    torch.distributions.Normal.rsample = rs
    orig_randint = torch.randint
    patch_randint(cfg, 1000, B, T)
    try:
        d = TD({k: torch.from_numpy(v) for k, v in data_np.items()}, batch_size=(B, T))
        d = ag.preprocess(d)
        ag._update_slow_target()
        if cfg.model.rep_loss == "dreamerpro":
            ag.ema_update()  # EMA encoder := online encoder, unit prototypes (as update 0 does)
        ag._cal_grad(d, (torch.from_numpy(init_np[0]), torch.from_numpy(init_np[1])))
    finally:
        torch.nn.functional.gumbel_softmax = orig_gs
        torch.distributions.Normal.rsample = orig_rs
        torch.randint = orig_randint
    out = {}
    named = dict(ag.named_parameters())
    for k in spec.shapes:
        g = named[k].grad
        flat = (torch.zeros_like(named[k]) if g is None else g).reshape(-1).numpy()
        idx = sample_idx(k, flat.size)
        out[f"g_{k}__n"] = np.asarray(np.linalg.norm(flat.astype(np.float64)))
        out[f"g_{k}__s"] = flat[idx]
    return out


def full_case(name, mods, TD):
    """One reference update() at a BASELINE size (tests/fullsize_io.py FULL: C2 walker B16 L64 H15, the C3 shard,
    C4 atari B32, C5 maze B16 L256 H25 deter 4096) on the inputs full_inputs() regenerates from the case name, with
    params_for() weights, model.warmup=0 and noise seed fullsize_io.SEED. Only outputs are stored, compactly: every
    metric, the posterior indices, deter columns, replay returns, ReturnEMA, imagined indices / deter columns /
    actions / returns of every ROW_STRIDE-th start row, and per parameter the norms of the step and of the second
    moment plus 32 sampled elements of the updated parameter and both LaProp moments."""
    cfg_name, ovr, obs, A, discrete, B, L, H = FULL[name]
    cfg = load_config(cfg_name, ["device=cpu"] + ovr + FULL_OVR)
    D = mods["world_model.dreamer"]

    class Sp:
        def __init__(s, shape):
            s.shape = shape

    class Spaces:
        def __init__(s, d):
            s.spaces = d

    act_space = Sp((A,))
    if discrete:
        act_space.discrete = True
    import copy
    ag = D.Dreamer(copy.deepcopy(cfg.model), Spaces({k: Sp(v) for k, v in obs.items()}), act_space)
    spec = Spec(cfg.model, obs, A, discrete)
    vals = params_for(spec.shapes, FULL_PARAM_SEED)
    with torch.no_grad():
        named = dict(ag.named_parameters())
        for k, v in vals.items():
            named[k].data.copy_(torch.from_numpy(v))
        for k, v in named.items():
            if k.startswith("_slow_value."):
                v.data.copy_(torch.from_numpy(vals["value." + k[len("_slow_value."):]]))
    data_np, init_np = full_inputs(name, spec.K, spec.S, spec.D)
    seq = NoiseSeq(L, H + 1, FULL_SEED, cfg.model.rep_loss == "dreamerpro")
    seq.discrete_act = discrete
    D.autocast = lambda **k: contextlib.nullcontext()
    orig_gs = torch.nn.functional.gumbel_softmax
    orig_rs = torch.distributions.Normal.rsample
    rec = {}

    def gs(logits, tau=1, hard=False, eps=1e-10, dim=-1):
        g = torch.from_numpy(seq.gumbel(tuple(logits.shape)))
        y_soft = ((logits + g) / tau).softmax(dim)
        index = y_soft.max(dim, keepdim=True)[1]
        return torch.zeros_like(logits).scatter_(dim, index, 1.0) - y_soft.detach() + y_soft

    def rs(self, sample_shape=torch.Size()):
        shape = self._extended_shape(sample_shape)
        return self.loc + torch.from_numpy(seq.normal(tuple(shape))) * self.scale

    def hook(obj, attr, key, many=False):
        orig = getattr(obj, attr)

        def w(*a, **k):
            r = orig(*a, **k)
            if many:
                rec.setdefault(key, []).append(r)
            else:
                rec.setdefault(key, r)
            return r

        setattr(obj, attr, w)

    hook(ag.rssm, "observe", "observe")
    hook(ag, "_imagine", "imagine")
    hook(ag, "_lambda_return", "lret", many=True)

    class Buf:
        def sample(self_):
            d = TD({k: torch.from_numpy(v) for k, v in data_np.items()}, batch_size=(B, L))
            return d, None, (torch.from_numpy(init_np[0]), torch.from_numpy(init_np[1]))

        def update(self_, index, stoch, deter):
            pass

    torch.nn.functional.gumbel_softmax = gs
    torch.distributions.Normal.rsample = rs
    try:
        mets = ag.update(Buf())
    finally:
        torch.nn.functional.gumbel_softmax = orig_gs
        torch.distributions.Normal.rsample = orig_rs
    assert seq.g == L + 1 + (H + 1) * (2 if discrete else 1), seq.g
    rs_ = FULL_STRIDE[name]
    out = {"meta_B": B, "meta_L": L, "meta_H": H, "meta_seed": FULL_SEED, "meta_param_seed": FULL_PARAM_SEED,
           "meta_row_stride": rs_}
    ps, pdet, _ = rec["observe"]
    dcol = max(1, spec.D // 8)
    out["post_idx"] = ps.argmax(-1).numpy().astype(np.uint8)
    out["post_deter"] = pdet.detach().numpy()[..., ::dcol].copy()
    ifeat, iact = rec["imagine"]  # (N, H1, F), (N, H1, A)
    SK = spec.SK
    out["imag_idx"] = ifeat[::rs_, :, :SK].reshape(-1, H + 1, spec.S, spec.K).argmax(-1).numpy().astype(np.uint8)
    out["imag_deter"] = ifeat[::rs_, :, SK::max(1, spec.D // 4)].numpy().copy()
    out["imag_action"] = (iact[::rs_].argmax(-1).numpy().astype(np.uint8) if discrete else iact[::rs_].numpy().copy())
    out["imag_ret"] = rec["lret"][0][::rs_, :, 0].numpy().copy()
    out["replay_ret"] = rec["lret"][1][..., 0].numpy().copy()
    for k, v in mets.items():
        out[f"m_{k}"] = np.asarray(float(v), np.float64)
    out["ema_vals"] = ag.return_ema.ema_vals.numpy().copy()
    named = dict(ag.named_parameters())
    for k in spec.shapes:
        p1 = named[k].detach().reshape(-1).numpy()
        p0 = vals[k].reshape(-1)
        st = ag._optimizer.state[named[k]]
        v = st["exp_avg_sq"].reshape(-1).numpy()
        idx = full_sample_idx(k, p1.size)
        out[f"dp_{k}__n"] = np.asarray(np.linalg.norm(p1.astype(np.float64) - p0.astype(np.float64)))
        out[f"v_{k}__n"] = np.asarray(np.linalg.norm(v.astype(np.float64)))
        out[f"v_{k}__max"] = np.asarray(float(np.abs(v).max()))
        out[f"p_{k}__s"] = p1[idx]
        out[f"m_{k}__s"] = st["exp_avg"].reshape(-1).numpy()[idx]
        out[f"v_{k}__s"] = v[idx]
    return out


def main():
    mods, TD = import_reference()
    torch.set_num_threads(8)
    args = sys.argv[1:]
    if args and args[0] == "full":  # python tests/golden/gen_golden.py full [case ...]
        for name in args[1:] or list(FULL):
            out = full_case(name, mods, TD)
            path = fixture_path(name)
            np.savez_compressed(path, **out)
            print(name, "->", path, os.path.getsize(path) // 1024, "KB")
        return
    only = args or list(CASES)
    lay_path = os.path.join(HERE, "optim_layout.json")
    layouts = json.load(open(lay_path)) if os.path.exists(lay_path) else {}
    for name in only:
        out, layouts[name] = run_case(name, mods, TD)
        out.update(grad_case(name, mods, TD))
        if CASES[name][0] == "dmc/walker_dreamer":
            out.update(video_case(name, mods, TD))
        path = os.path.join(HERE, f"{name}.npz")
        np.savez_compressed(path, **out)
        print(name, "->", path, os.path.getsize(path) // 1024, "KB")
    with open(lay_path, "w") as f:
        json.dump({k: layouts[k] for k in sorted(layouts)}, f, indent=1)


if __name__ == "__main__":
    main()
