"""fp32 PyTorch-CPU restatement of the reference hot path — TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Functional, op for op, with explicit parameters (keyed by the reference's state_dict names) and explicit
counter-based noise (oracle/noise.py). Every function cites the reference code it restates
(paths relative to /root/reference). Used as the parity checker for the HIP path and as the CPU baseline
timed by bench.py; pinned against tests/golden/*.npz (generated from the reference itself).
"""
from __future__ import annotations

import math
import re

import numpy as np
import torch
import torch.nn.functional as F

from . import noise as nz

# arithmetic type of the restatement: float32 (the reference's) everywhere in the tests; tools/grad_attrib.py sets
# float64 to get the exact-arithmetic answer the f32 results are each an approximation of (inputs that the reference
# forms in f32 — images / 255, the augmentation's grid_sample, Philox noise — stay f32 values)
DT = torch.float32

# --------------------------------------------------------------------------------------------------------
# distributions (world_model/distributions.py)
# --------------------------------------------------------------------------------------------------------


def symlog(x):  # distributions.py:8-9
    return torch.sign(x) * torch.log1p(torch.abs(x))


def symexp(x):  # distributions.py:12-13
    return torch.sign(x) * torch.expm1(torch.abs(x))


def unimix_logits(logits, unimix):
    """OneHotDist.__init__ (distributions.py:17-22) + Categorical logit normalisation (torch)."""
    probs = F.softmax(logits.to(DT), dim=-1)
    uniform = unimix / probs.shape[-1]
    probs = probs * (1.0 - unimix) + torch.ones_like(probs, dtype=DT) * uniform
    lg = torch.log(probs)
    return lg - lg.logsumexp(dim=-1, keepdim=True)


def st_gumbel_sample(norm_logits, g, force=None):
    """OneHotDist.rsample (distributions.py:32-33) = F.gumbel_softmax(hard=True) with injected gumbel g.

    force (tests only, teacher forcing at near-ties): (site, index) integer arrays; the hard sample at `site` (a
    tuple of leading indices, e.g. (rows, latents)) takes `index` instead of the argmax. The soft part, and so the
    straight-through gradient, is untouched."""
    y_soft = ((norm_logits + g) / 1.0).softmax(-1)
    index = y_soft.max(-1, keepdim=True)[1]
    if force is not None:
        site, k = force
        index[tuple(torch.as_tensor(np.asarray(a), dtype=torch.long) for a in site) + (0,)] = \
            torch.as_tensor(np.asarray(k), dtype=torch.long)
    y_hard = torch.zeros_like(norm_logits).scatter_(-1, index, 1.0)
    return y_hard - y_soft.detach() + y_soft


def cat_entropy(norm_logits):
    """Categorical.entropy (torch) on normalised logits, summed over the Independent dim by callers."""
    min_real = torch.finfo(norm_logits.dtype).min
    lg = torch.clamp(norm_logits, min=min_real)
    p = F.softmax(norm_logits, dim=-1)
    return -(lg * p).sum(-1)


def onehot_mode(norm_logits):  # distributions.py:25-29
    m = F.one_hot(torch.argmax(norm_logits, axis=-1), norm_logits.shape[-1])
    return m.detach() + norm_logits - norm_logits.detach()


def onehot_log_prob(norm_logits, value):  # torch OneHotCategorical.log_prob
    idx = value.max(-1)[1]
    return norm_logits.gather(-1, idx.unsqueeze(-1)).squeeze(-1)


def kl_cat(left, right):  # distributions.py:266-271
    lp_l = torch.log_softmax(left, -1)
    lp_r = torch.log_softmax(right, -1)
    p = torch.softmax(left, -1)
    return (p * (lp_l - lp_r)).sum(-1)


def twohot_bins(bin_num=255):  # distributions.py:242-251
    if bin_num % 2 == 1:
        half = torch.linspace(-20, 0, (bin_num - 1) // 2 + 1, dtype=DT)
        half = symexp(half)
        return torch.concatenate([half, -half[:-1].flip(dims=(0,))], 0)
    half = symexp(torch.linspace(-20, 0, bin_num // 2, dtype=DT))
    return torch.concatenate([half, -half.flip(dims=(0,))], 0)


def twohot_mode(logits, bins):  # TwoHot.mode, distributions.py:78-98
    probs = F.softmax(logits.to(DT), dim=-1)
    n = logits.shape[-1]
    if n % 2 == 1:
        m = (n - 1) // 2
        p1, p2, p3 = probs[..., :m], probs[..., m:m + 1], probs[..., m + 1:]
        b1, b2, b3 = bins[..., :m], bins[..., m:m + 1], bins[..., m + 1:]
        return (p2 * b2).sum(-1, keepdim=True) + ((p1 * b1).flip(dims=(-1,)) + (p3 * b3)).sum(-1, keepdim=True)
    p1, p2 = probs[..., :n // 2], probs[..., n // 2:]
    b1, b2 = bins[..., :n // 2], bins[..., n // 2:]
    return ((p1 * b1).flip(dims=(-1,)) + (p2 * b2)).sum(-1, keepdim=True)


def twohot_log_prob(logits, bins, target):  # TwoHot.log_prob, distributions.py:100-129
    logits = logits.to(DT)
    target = target.squeeze(-1)
    ts = target.detach()
    nb = len(bins)
    below = (bins <= ts.unsqueeze(-1)).to(torch.int32).sum(-1) - 1
    above = nb - (bins > ts.unsqueeze(-1)).to(torch.int32).sum(-1)
    below = torch.clamp(below, 0, nb - 1)
    above = torch.clamp(above, 0, nb - 1)
    equal = below == above
    one = torch.tensor(1.0, dtype=DT)
    d_below = torch.where(equal, one, (bins[below] - ts).abs())
    d_above = torch.where(equal, one, (bins[above] - ts).abs())
    total = d_below + d_above
    w_below = d_above / total
    w_above = d_below / total
    target_dist = (F.one_hot(below, nb).to(DT) * w_below.unsqueeze(-1)
                   + F.one_hot(above, nb).to(DT) * w_above.unsqueeze(-1))
    log_pred = logits - torch.logsumexp(logits, dim=-1, keepdim=True)
    return (target_dist * log_pred).sum(-1)


def bernoulli_log_prob(logits, value):  # torchd.Bernoulli(logits).log_prob, summed by Independent(…, 1)
    return (-F.binary_cross_entropy_with_logits(logits.to(DT), value, reduction="none")).sum(-1)


def bounded_normal_params(x, min_std, max_std):  # distributions.py:217-222
    mean, std = torch.chunk(x, 2, dim=-1)
    std = (max_std - min_std) * torch.sigmoid(std + 2.0) + min_std
    return torch.tanh(mean.to(DT)), std.to(DT)


def normal_log_prob(loc, scale, value):  # torchd.Normal.log_prob, summed by Independent
    var = scale ** 2
    return (-((value - loc) ** 2) / (2 * var) - scale.log() - math.log(math.sqrt(2 * math.pi))).sum(-1)


def normal_entropy(scale):  # torchd.Normal.entropy, summed by Independent
    return (0.5 + 0.5 * math.log(2 * math.pi) + torch.log(scale)).sum(-1)


# --------------------------------------------------------------------------------------------------------
# layers (world_model/networks.py, world_model/rssm.py)
# --------------------------------------------------------------------------------------------------------


def rms(x, w):  # nn.RMSNorm(eps=1e-4)
    return F.rms_norm(x, (x.shape[-1],), w, 1e-4)


def block_linear(x, w, b, blocks):  # BlockLinear.forward, networks.py:43-56
    bs = x.shape[:-1]
    x = x.view(*bs, blocks, x.shape[-1] // blocks)
    x = torch.einsum("...gi,oig->...go", x, w)
    return x.reshape(*bs, w.shape[0] * blocks) + b


def conv_same(x, w, b):  # Conv2dSamePad.forward, networks.py:62-85 (stride 1, dilation 1)
    k = w.shape[-1]
    pad = max(k - 1, 0)
    x = F.pad(x, [pad // 2, pad - pad // 2, pad // 2, pad - pad // 2])
    return F.conv2d(x, w, b)


def rms2d(x, w):  # RMSNorm2D.forward, networks.py:94-96
    return rms(x.permute(0, 2, 3, 1), w).permute(0, 3, 1, 2)


# --------------------------------------------------------------------------------------------------------
# model description
# --------------------------------------------------------------------------------------------------------


class Spec:
    """Static dims + parameter-name table of a Dreamer built from `config.model` (dreamer.py:23-233)."""

    def __init__(self, mcfg, obs_shapes: dict, act_dim: int, act_discrete: bool):
        self.cfg = mcfg
        r = mcfg.rssm
        self.S, self.K, self.D, self.U, self.G = int(r.stoch), int(r.discrete), int(r.deter), int(r.hidden), int(r.blocks)
        self.SK = self.S * self.K
        self.F = self.SK + self.D
        self.unimix = float(r.unimix_ratio)
        self.A = int(act_dim)
        self.discrete = bool(act_discrete)
        self.rep_loss = str(mcfg.rep_loss)
        ad = mcfg.actor.dist  # dreamer.py:73-82 resolves config.actor.dist to its cont/disc branch
        self.actor_dist = ad if "name" in ad else (ad.disc if act_discrete else ad.cont)
        enc = mcfg.encoder
        excl = ("is_first", "is_last", "is_terminal", "reward")
        shp = {k: tuple(v) for k, v in obs_shapes.items() if k not in excl and not k.startswith("log_")}
        self.cnn_keys = [k for k, v in shp.items() if len(v) == 3 and re.match(enc.cnn_keys, k)]
        self.mlp_keys = [k for k, v in shp.items() if len(v) in (1, 2) and re.match(enc.mlp_keys, k)]
        self.obs_shapes = shp
        p = {}
        E = 0
        ei = 0
        if self.cnn_keys:
            c = enc.cnn
            self.enc_depths = [int(c.depth) * int(m) for m in c.mults]
            self.ksz = int(c.kernel_size)
            ch = sum(shp[k][-1] for k in self.cnn_keys)
            h, w = shp[self.cnn_keys[0]][:2]
            for i, d in enumerate(self.enc_depths):
                p[f"encoder.encoders.{ei}.layers.{4 * i}.weight"] = (d, ch, self.ksz, self.ksz)
                p[f"encoder.encoders.{ei}.layers.{4 * i}.bias"] = (d,)
                p[f"encoder.encoders.{ei}.layers.{4 * i + 2}.weight"] = (d,)
                ch = d
                h, w = h // 2, w // 2
            E += ch * h * w
            self.cnn_enc_idx = ei
            ei += 1
        if self.mlp_keys:
            c = enc.mlp
            inp = sum(sum(shp[k]) for k in self.mlp_keys)
            for i in range(int(c.layers)):
                p[f"encoder.encoders.{ei}.layers.{c.name}_linear{i}.weight"] = (int(c.units), inp)
                p[f"encoder.encoders.{ei}.layers.{c.name}_linear{i}.bias"] = (int(c.units),)
                p[f"encoder.encoders.{ei}.layers.{c.name}_norm{i}.weight"] = (int(c.units),)
                inp = int(c.units)
            E += int(c.units)
            self.mlp_enc_idx = ei
            ei += 1
        self.E = E
        D, U, G, SK, A = self.D, self.U, self.G, self.SK, self.A
        pre = "rssm._deter_net."
        for nm, i_dim in (("_dyn_in0", D), ("_dyn_in1", SK), ("_dyn_in2", A)):
            p[pre + nm + ".0.weight"] = (U, i_dim)
            p[pre + nm + ".0.bias"] = (U,)
            p[pre + nm + ".1.weight"] = (U,)
        in_ch = (3 * U + D // G) * G
        self.dyn_layers = int(r.dyn_layers)
        for i in range(self.dyn_layers):
            p[pre + f"_dyn_hid.dyn_hid_{i}.weight"] = (D // G, in_ch // G, G)
            p[pre + f"_dyn_hid.dyn_hid_{i}.bias"] = (D,)
            p[pre + f"_dyn_hid.norm_{i}.weight"] = (D,)
            in_ch = D
        p[pre + "_dyn_gru.weight"] = (3 * D // G, in_ch // G, G)
        p[pre + "_dyn_gru.bias"] = (3 * D,)
        self.obs_layers, self.img_layers = int(r.obs_layers), int(r.img_layers)
        inp = D + E
        for i in range(self.obs_layers):
            p[f"rssm._obs_net.obs_net_{i}.weight"] = (U, inp)
            p[f"rssm._obs_net.obs_net_{i}.bias"] = (U,)
            p[f"rssm._obs_net.obs_net_n_{i}.weight"] = (U,)
            inp = U
        p["rssm._obs_net.obs_net_logit.weight"] = (SK, inp)
        p["rssm._obs_net.obs_net_logit.bias"] = (SK,)
        inp = D
        for i in range(self.img_layers):
            p[f"rssm._img_net.img_net_{i}.weight"] = (U, inp)
            p[f"rssm._img_net.img_net_{i}.bias"] = (U,)
            p[f"rssm._img_net.img_net_n_{i}.weight"] = (U,)
            inp = U
        p["rssm._img_net.img_net_logit.weight"] = (SK, inp)
        p["rssm._img_net.img_net_logit.bias"] = (SK,)
        Fd = self.F
        act_out = A if self.discrete else 2 * A
        self.heads = {}
        for head, hc, out in (("reward", mcfg.reward, int(mcfg.reward.shape[0])), ("cont", mcfg.cont, 1),
                              ("actor", mcfg.actor, act_out), ("value", mcfg.critic, int(mcfg.critic.shape[0]))):
            self.heads[head] = (str(hc.name), int(hc.layers))
            inp = Fd
            for i in range(int(hc.layers)):
                p[f"{head}.mlp.layers.{hc.name}_linear{i}.weight"] = (int(hc.units), inp)
                p[f"{head}.mlp.layers.{hc.name}_linear{i}.bias"] = (int(hc.units),)
                p[f"{head}.mlp.layers.{hc.name}_norm{i}.weight"] = (int(hc.units),)
                inp = int(hc.units)
            p[f"{head}.last.weight"] = (out, inp)
            p[f"{head}.last.bias"] = (out,)
        self.slow_names = {}
        for k in list(p):
            if k.startswith("value."):
                self.slow_names[k] = "_slow_value." + k[len("value."):]
        self.ema_names = {}
        if self.rep_loss in ("r2dreamer", "infonce"):
            p["prj.w.weight"] = (E, Fd)
        elif self.rep_loss == "dreamerpro":  # dreamer.py:131-162
            dpc = mcfg.dreamer_pro
            Kp, Pd = int(dpc.num_prototypes), int(dpc.proto_dim)
            enc_names = [k for k in p if k.startswith("encoder.")]
            p["_prototypes"] = (Kp, Pd)
            p["obs_proj.weight"] = (Pd, E)
            p["obs_proj.bias"] = (Pd,)
            p["feat_proj.weight"] = (Pd, Fd)
            p["feat_proj.bias"] = (Pd,)
            self.ema_names = {k: "_ema_" + k for k in enc_names}
            self.ema_names.update({"obs_proj.weight": "_ema_obs_proj.weight", "obs_proj.bias": "_ema_obs_proj.bias"})
        elif self.rep_loss == "dreamer":
            dec = mcfg.decoder
            dexcl = ("is_first", "is_last", "is_terminal")
            dshp = {k: tuple(v) for k, v in obs_shapes.items() if k not in dexcl}
            self.dec_cnn_keys = [k for k, v in dshp.items() if len(v) == 3 and re.match(dec.cnn_keys, k)]
            self.dec_mlp_keys = [k for k, v in dshp.items() if len(v) in (1, 2) and re.match(dec.mlp_keys, k)]
            if self.dec_cnn_keys:
                c = dec.cnn
                depths = [int(c.depth) * int(m) for m in c.mults]
                self.dec_depths = depths
                hw = dshp[self.dec_cnn_keys[0]][:2]
                f = 2 ** len(depths)
                self.dec_min = (hw[0] // f, hw[1] // f, depths[-1])
                u = int(np.prod(self.dec_min))
                g = int(c.bspace)
                self.dec_bspace = g
                self.dec_out_ch = sum(dshp[k][-1] for k in self.dec_cnn_keys)
                kk = int(c.kernel_size)
                p["decoder._cnn.sp0.weight"] = (u // g, D // g, g)
                p["decoder._cnn.sp0.bias"] = (u,)
                p["decoder._cnn.sp1.0.weight"] = (2 * int(c.units), SK)
                p["decoder._cnn.sp1.0.bias"] = (2 * int(c.units),)
                p["decoder._cnn.sp1.1.weight"] = (2 * int(c.units),)
                p["decoder._cnn.sp2.weight"] = (u, 2 * int(c.units))
                p["decoder._cnn.sp2.bias"] = (u,)
                p["decoder._cnn.sp_norm.0.weight"] = (depths[-1],)
                ch = depths[-1]
                li = 0
                self.dec_layers = []
                for d in reversed(depths[:-1]):
                    p[f"decoder._cnn.layers.{li + 1}.weight"] = (d, ch, kk, kk)
                    p[f"decoder._cnn.layers.{li + 1}.bias"] = (d,)
                    p[f"decoder._cnn.layers.{li + 2}.weight"] = (d,)
                    self.dec_layers.append((li + 1, li + 2))
                    ch = d
                    li += 4
                p[f"decoder._cnn.layers.{li + 1}.weight"] = (self.dec_out_ch, ch, kk, kk)
                p[f"decoder._cnn.layers.{li + 1}.bias"] = (self.dec_out_ch,)
                self.dec_last = li + 1
            if self.dec_mlp_keys:
                c = dec.mlp
                inp = D + SK
                for i in range(int(c.layers)):
                    p[f"decoder._mlp.mlp.layers.{c.name}_linear{i}.weight"] = (int(c.units), inp)
                    p[f"decoder._mlp.mlp.layers.{c.name}_linear{i}.bias"] = (int(c.units),)
                    p[f"decoder._mlp.mlp.layers.{c.name}_norm{i}.weight"] = (int(c.units),)
                    inp = int(c.units)
                out = sum(sum(dshp[k]) for k in self.dec_mlp_keys)
                p["decoder._mlp.last.weight"] = (out, inp)
                p["decoder._mlp.last.bias"] = (out,)
                self.dec_mlp_name = str(c.name)
                self.dec_mlp_layers = int(c.layers)
                self.dec_mlp_split = [sum(dshp[k]) for k in self.dec_mlp_keys]
        else:
            raise NotImplementedError(self.rep_loss)
        self.shapes = p
        self.trainable = [k for k in p]  # _slow_value.* added separately (not trainable)


# --------------------------------------------------------------------------------------------------------
# forward pieces
# --------------------------------------------------------------------------------------------------------


def random_translate(img, shifts, pad, bilinear):
    """Dreamer.random_translate (dreamer.py:845-880) on (B, T, H, W, C) images with given integer shifts (B, T, 2)
    = (x, y) in [0, 2 pad]: out[y][x] = in[clamp(y + sy - pad)][clamp(x + sx - pad)]. The reference samples the
    replicate-padded image with grid_sample at exactly those pixel centres; bilinear mode does so through float
    grid arithmetic, whose last-bit weights (|d| ~ 6e-8) are reproduced here (torch's own grid_sample) so the oracle
    tracks the reference's gradients to the golden tolerance. The HIP kernel restates that f32 arithmetic
    (sd_random_translate, bilinear = 1) and is pinned bit-exact against this function."""
    B, T, H, W, C = img.shape
    x = F.pad(img.reshape(B * T, H, W, C).permute(0, 3, 1, 2), (pad, pad, pad, pad), mode="replicate")
    Hp, Wp = H + 2 * pad, W + 2 * pad
    if not bilinear:
        ys = torch.arange(H)[None, :] + shifts.reshape(B * T, 2)[:, 1:2]
        xs = torch.arange(W)[None, :] + shifts.reshape(B * T, 2)[:, 0:1]
        out = x[torch.arange(B * T)[:, None, None], :, ys[:, :, None], xs[:, None, :]]  # (BT, H, W, C)
        return out.reshape(B, T, H, W, C)
    gy = torch.linspace(-1.0 + 1.0 / Hp, 1.0 - 1.0 / Hp, Hp)[:H]
    gx = torch.linspace(-1.0 + 1.0 / Wp, 1.0 - 1.0 / Wp, Wp)[:W]
    grid = torch.stack([gx[None, :].expand(H, W), gy[:, None].expand(H, W)], -1)[None]  # (1, H, W, 2): (x, y)
    off = shifts.reshape(B * T, 1, 1, 2).float() * 2.0 / torch.tensor([Wp, Hp], dtype=torch.float32)
    out = F.grid_sample(x.float(), grid + off, mode="bilinear", padding_mode="zeros", align_corners=False)
    return out.permute(0, 2, 3, 1).reshape(B, T, H, W, C).to(img.dtype)


class Oracle:
    """Dreamer hot path on CPU. `P` maps reference state_dict names to fp32 tensors (leafs for trainables)."""

    def __init__(self, spec: Spec, P: dict):
        self.s = spec
        self.P = P
        # teacher forcing (tests only): {(kind, stream, step): (site arrays, indices)} for kind "obs" (posterior
        # sample of observe step `step` on noise stream `stream`), "img" (prior sample of img_step `step`) and "act"
        # (actor sample at imagined step `step`); see tests/test_gpu_fullsize.py
        self.force = {}
        c = spec.cfg
        self.bins = twohot_bins(int(c.critic.dist.bin_num))
        self.rbins = twohot_bins(int(c.reward.dist.bin_num))

    # ---- encoder (networks.py:99-141, 192-234, 313-336)
    def encode(self, data, P=None):  # P: a parameter table with the encoder.* names (the EMA encoder's view)
        s, P = self.s, (P or self.P)
        outs = []
        if s.cnn_keys:
            obs = torch.cat([data[k] for k in s.cnn_keys], -1)
            obs = obs - 0.5
            x = obs.reshape(-1, *obs.shape[-3:]).permute(0, 3, 1, 2)
            pre = f"encoder.encoders.{s.cnn_enc_idx}.layers."
            for i in range(len(s.enc_depths)):
                x = conv_same(x, P[pre + f"{4 * i}.weight"], P[pre + f"{4 * i}.bias"])
                x = F.max_pool2d(x, 2, 2)
                x = rms2d(x, P[pre + f"{4 * i + 2}.weight"])
                x = F.silu(x)
            x = x.reshape(x.shape[0], -1)
            outs.append(x.reshape(*obs.shape[:-3], x.shape[-1]))
        if s.mlp_keys:
            x = torch.cat([data[k] for k in s.mlp_keys], -1)
            c = s.cfg.encoder.mlp
            if bool(c.symlog_inputs):
                x = symlog(x)
            pre = f"encoder.encoders.{s.mlp_enc_idx}.layers.{c.name}"
            for i in range(int(c.layers)):
                x = F.silu(rms(F.linear(x, P[f"{pre}_linear{i}.weight"], P[f"{pre}_linear{i}.bias"]),
                               P[f"{pre}_norm{i}.weight"]))
            outs.append(x)
        return outs[0] if len(outs) == 1 else torch.cat(outs, -1)

    # ---- RSSM (rssm.py)
    def deter_step(self, stoch, deter, action, P=None):  # Deter.forward, rssm.py:36-75
        s = self.s
        P = P or self.P
        pre = "rssm._deter_net."
        B = action.shape[0]
        stoch = stoch.reshape(B, -1)
        action = action / torch.clip(torch.abs(action), min=1.0).detach()

        def inp(nm, x):
            return F.silu(rms(F.linear(x, P[pre + nm + ".0.weight"], P[pre + nm + ".0.bias"]), P[pre + nm + ".1.weight"]))

        x0, x1, x2 = inp("_dyn_in0", deter), inp("_dyn_in1", stoch), inp("_dyn_in2", action)
        x = torch.cat([x0, x1, x2], -1).unsqueeze(-2).expand(-1, s.G, -1)
        x = torch.cat([deter.reshape(B, s.G, -1), x], -1).reshape(B, -1)
        for i in range(s.dyn_layers):
            x = block_linear(x, P[pre + f"_dyn_hid.dyn_hid_{i}.weight"], P[pre + f"_dyn_hid.dyn_hid_{i}.bias"], s.G)
            x = F.silu(rms(x, P[pre + f"_dyn_hid.norm_{i}.weight"]))
        x = block_linear(x, P[pre + "_dyn_gru.weight"], P[pre + "_dyn_gru.bias"], s.G)
        gates = torch.chunk(x.reshape(B, s.G, -1), 3, dim=-1)
        reset, cand, update = (g.reshape(B, -1) for g in gates)
        reset = torch.sigmoid(reset)
        cand = torch.tanh(reset * cand)
        update = torch.sigmoid(update - 1)
        return update * cand + (1 - update) * deter

    def obs_logit(self, deter, embed, P=None):  # rssm.py:106-117,170-173
        s = self.s
        P = P or self.P
        x = torch.cat([deter, embed], -1)
        for i in range(s.obs_layers):
            x = F.silu(rms(F.linear(x, P[f"rssm._obs_net.obs_net_{i}.weight"], P[f"rssm._obs_net.obs_net_{i}.bias"]),
                           P[f"rssm._obs_net.obs_net_n_{i}.weight"]))
        x = F.linear(x, P["rssm._obs_net.obs_net_logit.weight"], P["rssm._obs_net.obs_net_logit.bias"])
        return x.reshape(*x.shape[:-1], s.S, s.K)

    def img_logit(self, deter, P=None):  # rssm.py:119-130,189-195
        s = self.s
        P = P or self.P
        x = deter
        for i in range(s.img_layers):
            x = F.silu(rms(F.linear(x, P[f"rssm._img_net.img_net_{i}.weight"], P[f"rssm._img_net.img_net_{i}.bias"]),
                           P[f"rssm._img_net.img_net_n_{i}.weight"]))
        x = F.linear(x, P["rssm._img_net.img_net_logit.weight"], P["rssm._img_net.img_net_logit.bias"])
        return x.reshape(*x.shape[:-1], s.S, s.K)

    def sample_stoch(self, logit, g, force=None):  # get_dist(logit).rsample(), rssm.py:219-220 + distributions.py:32-33
        return st_gumbel_sample(unimix_logits(logit, self.s.unimix), g, force)

    def observe(self, embed, action, initial, reset, seed, row_offset=0, stream=nz.STREAM_OBS):  # rssm.py:140-156
        s = self.s
        L = action.shape[1]
        B = action.shape[0]
        stoch, deter = initial
        stochs, deters, logits = [], [], []
        for i in range(L):
            rs = reset[:, i]
            m = rs.reshape(B, *([1] * (stoch.dim() - 1)))
            stoch = torch.where(m, torch.zeros_like(stoch), stoch)  # rssm.py:161-165
            deter = torch.where(rs.reshape(B, 1), torch.zeros_like(deter), deter)
            act = torch.where(rs.reshape(B, 1), torch.zeros_like(action[:, i]), action[:, i])
            deter = self.deter_step(stoch, deter, act)
            logit = self.obs_logit(deter, embed[:, i])
            g = torch.from_numpy(nz.gumbel_block(seed, stream, i, B, row_offset, s.SK)).reshape(B, s.S, s.K)
            stoch = self.sample_stoch(logit, g, self.force.get(("obs", stream, i)))
            stochs.append(stoch)
            deters.append(deter)
            logits.append(logit)
        return torch.stack(stochs, 1), torch.stack(deters, 1), torch.stack(logits, 1)

    def get_feat(self, stoch, deter):  # rssm.py:211-217
        return torch.cat([stoch.reshape(*stoch.shape[:-2], self.s.SK), deter], -1)

    # ---- heads (networks.py:339-377)
    def head_logits(self, head, x, P=None):
        P = P or self.P
        pre = "_slow_value" if head == "slow_value" else head
        name, layers = self.s.heads["value" if head == "slow_value" else head]
        for i in range(layers):
            x = F.silu(rms(F.linear(x, P[f"{pre}.mlp.layers.{name}_linear{i}.weight"],
                                    P[f"{pre}.mlp.layers.{name}_linear{i}.bias"]),
                           P[f"{pre}.mlp.layers.{name}_norm{i}.weight"]))
        return F.linear(x, P[f"{pre}.last.weight"], P[f"{pre}.last.bias"])

    def actor_sample(self, logits, seed, step, row_offset, stream=nz.STREAM_ACT):
        """frozen actor rsample (dreamer.py:684): bounded_normal or onehot."""
        s = self.s
        N = logits.shape[0]
        if s.discrete:
            nl = unimix_logits(logits, float(s.actor_dist.unimix_ratio))
            g = torch.from_numpy(nz.gumbel_block(seed, stream, step, N, row_offset, s.A))
            return st_gumbel_sample(nl, g, self.force.get(("act", stream, step)))
        loc, scale = bounded_normal_params(logits, float(s.actor_dist.min_std), float(s.actor_dist.max_std))
        eps = torch.from_numpy(nz.normal_block(seed, stream, step, N, row_offset, s.A))
        return loc + eps * scale

    @torch.no_grad()
    def act(self, obs, state, seed, step=0, eval=False):
        """Dreamer.act (dreamer.py:330-357; the frozen modules share the trained weights): encoder on the (B, *)
        observation, RSSM.obs_step (rssm.py:158-178: is_first resets the carried state), actor mode or rsample.
        Noise: posterior sample STREAM_POLICY, action sample STREAM_POLICY_ACT."""
        s = self.s
        data = {k: v.unsqueeze(1) for k, v in obs.items() if k != "is_first"}
        if "image" in data and data["image"].dtype == torch.uint8:
            data["image"] = (data["image"].float() / 255.0).to(DT)  # Dreamer.preprocess, dreamer.py:710-713
        embed = self.encode(data)[:, 0]
        B = embed.shape[0]
        rs = obs["is_first"].reshape(B)
        stoch = torch.where(rs.reshape(B, 1, 1), torch.zeros_like(state["stoch"]), state["stoch"])
        deter = torch.where(rs.reshape(B, 1), torch.zeros_like(state["deter"]), state["deter"])
        act = torch.where(rs.reshape(B, 1), torch.zeros_like(state["prev_action"]), state["prev_action"])
        deter = self.deter_step(stoch, deter, act)
        logit = self.obs_logit(deter, embed)
        g = torch.from_numpy(nz.gumbel_block(seed, nz.STREAM_POLICY, step, B, 0, s.SK)).reshape(B, s.S, s.K)
        stoch = self.sample_stoch(logit, g)
        logits = self.head_logits("actor", self.get_feat(stoch, deter))
        if eval:
            if s.discrete:
                action = F.one_hot(logits.argmax(-1), s.A).to(DT)
            else:
                action = torch.tanh(logits[:, :s.A])
        else:
            action = self.actor_sample(logits, seed, step, 0, nz.STREAM_POLICY_ACT)
        return action, {"stoch": stoch, "deter": deter, "prev_action": action}

    @torch.no_grad()
    def imagine(self, start, horizon, seed, row_offset=0, rec=None):  # Dreamer._imagine, dreamer.py:673-692
        """rec (tests only): if a dict, collects the per-step actor logits and prior logits (near-tie margins)."""
        P = {k: v.detach() for k, v in self.P.items()}
        stoch, deter = start
        N = deter.shape[0]
        feats, actions = [], []
        for t in range(horizon):
            feat = self.get_feat(stoch, deter)
            alogit = self.head_logits("actor", feat, P)
            action = self.actor_sample(alogit, seed, t, row_offset)
            feats.append(feat)
            actions.append(action)
            if rec is not None:
                rec.setdefault("imag_actor_logit", []).append(alogit)
            if t == horizon - 1:
                break  # the last img_step's output is discarded by the reference (dreamer.py:688)
            deter = self.deter_step(stoch, deter, action, P)
            g = torch.from_numpy(nz.gumbel_block(seed, nz.STREAM_IMG, t, N, row_offset, self.s.SK))
            ilogit = self.img_logit(deter, P)
            stoch = self.sample_stoch(ilogit, g.reshape(N, self.s.S, self.s.K), self.force.get(("img", nz.STREAM_IMG, t)))
            if rec is not None:
                rec.setdefault("imag_prior_logit", []).append(ilogit)
        return torch.stack(feats, 1), torch.stack(actions, 1)


@torch.no_grad()
def lambda_return(last, term, reward, value, boot, disc, lamb):  # Dreamer._lambda_return, dreamer.py:694-707
    live = (1 - term.to(DT))[:, 1:] * disc
    cont = (1 - last.to(DT))[:, 1:] * lamb
    interm = reward[:, 1:] + (1 - cont) * live * boot[:, 1:]
    out = [boot[:, -1]]
    for i in reversed(range(live.shape[1])):
        out.append(interm[:, i] + live[:, i] * cont[:, i] * out[-1])
    return torch.stack(list(reversed(out))[:-1], 1)


def return_ema(ema_vals, x, alpha=1e-2):  # ReturnEMA.__call__, networks.py:416-422 (mutates ema_vals)
    q = torch.quantile(torch.flatten(x.detach()), torch.tensor([0.05, 0.95], dtype=x.dtype))
    ema_vals.copy_(alpha * q.detach() + (1 - alpha) * ema_vals)
    scale = torch.clip(ema_vals[1] - ema_vals[0], min=1.0)
    return ema_vals[0].detach(), scale.detach()


def tensorstats(t, prefix):  # tools.py:275-281
    return {f"{prefix}_mean": torch.mean(t), f"{prefix}_std": torch.std(t),
            f"{prefix}_min": torch.min(t), f"{prefix}_max": torch.max(t)}


# --------------------------------------------------------------------------------------------------------
# the update (dreamer.py:402-671) + optimiser (utils/optim)
# --------------------------------------------------------------------------------------------------------


class OracleAgent:
    """Stateful CPU agent: params, slow critic, ReturnEMA, LaProp state, LR schedule."""

    def __init__(self, spec: Spec, params: dict):
        self.s = spec
        self.P = {}
        for k in spec.shapes:
            self.P[k] = torch.tensor(params[k], dtype=DT).requires_grad_(True)
        for k, sk in spec.slow_names.items():
            v = params.get(sk, params[k])
            self.P[sk] = torch.tensor(v, dtype=DT)
        for k, ek in spec.ema_names.items():  # DreamerPro's EMA encoder / projection (not trainable)
            self.P[ek] = torch.tensor(params.get(ek, params[k]), dtype=DT)
        self.ema_updates = 0
        self.ema_vals = torch.zeros(2, dtype=DT)
        self.model = Oracle(spec, self.P)
        c = spec.cfg
        self.lr0 = float(c.lr)
        self.warmup = int(c.warmup)
        self.betas = (float(c.beta1), float(c.beta2))
        self.eps = float(c.eps)
        self.agc, self.pmin = float(c.agc), float(c.pmin)
        self.opt_step = 0  # LambdaLR last_epoch
        self.state = {}
        self.slow_updates = 0
        self.loss_scales = dict(c.loss_scales)
        if spec.rep_loss == "dreamer":
            rec = self.loss_scales.pop("recon")
            for k in spec.dec_cnn_keys + spec.dec_mlp_keys:
                self.loss_scales[k] = rec

    def lr(self):  # LambdaLR(lr_lambda) with warmup, dreamer.py:214-225
        if self.warmup:
            return self.lr0 * min(1.0, (self.opt_step + 1) / self.warmup)
        return self.lr0

    def trainable(self):
        return [self.P[k] for k in self.s.shapes]

    def update_slow_target(self):  # dreamer.py:242-249 (slow_target_update = 1)
        mix = float(self.s.cfg.slow_target_fraction)
        upd = int(self.s.cfg.slow_target_update)
        if self.slow_updates % upd == 0:
            with torch.no_grad():
                for k, sk in self.s.slow_names.items():
                    self.P[sk].copy_(mix * self.P[k].data + (1 - mix) * self.P[sk].data)
        self.slow_updates += 1

    def decode_losses(self, data, post_stoch, post_deter):  # MultiDecoder + MSEDist/SymlogDist, networks.py:144-310
        s, P, M = self.s, self.P, self.model
        out = {}
        if s.dec_cnn_keys:
            BT = post_deter.shape[:-1]
            x0 = post_deter.reshape(-1, s.D)
            x1 = post_stoch.reshape(-1, s.SK)
            H, W, C = s.dec_min
            x0 = block_linear(x0, P["decoder._cnn.sp0.weight"], P["decoder._cnn.sp0.bias"], s.dec_bspace)
            x0 = x0.reshape(-1, s.dec_bspace, H, W, C // s.dec_bspace).permute(0, 2, 3, 1, 4).reshape(-1, H, W, C)
            x1 = F.silu(rms(F.linear(x1, P["decoder._cnn.sp1.0.weight"], P["decoder._cnn.sp1.0.bias"]),
                            P["decoder._cnn.sp1.1.weight"]))
            x1 = F.linear(x1, P["decoder._cnn.sp2.weight"], P["decoder._cnn.sp2.bias"]).reshape(-1, H, W, C)
            x = F.silu(rms(x0 + x1, P["decoder._cnn.sp_norm.0.weight"]))
            x = x.permute(0, 3, 1, 2)
            for ci, ni in s.dec_layers:
                x = F.interpolate(x, scale_factor=2, mode="nearest")
                x = conv_same(x, P[f"decoder._cnn.layers.{ci}.weight"], P[f"decoder._cnn.layers.{ci}.bias"])
                x = F.silu(rms2d(x, P[f"decoder._cnn.layers.{ni}.weight"]))
            x = F.interpolate(x, scale_factor=2, mode="nearest")
            x = conv_same(x, P[f"decoder._cnn.layers.{s.dec_last}.weight"], P[f"decoder._cnn.layers.{s.dec_last}.bias"])
            x = torch.sigmoid(x.permute(0, 2, 3, 1))
            x = x.reshape(*BT, *x.shape[1:])
            splits = torch.split(x, [s.obs_shapes[k][-1] for k in s.dec_cnn_keys], -1)
            for k, mode in zip(s.dec_cnn_keys, splits):
                dist = (mode.to(DT) - data[k]) ** 2  # MSEDist(agg=sum), distributions.py:146-155
                out[k] = torch.mean(dist.sum(list(range(dist.dim()))[2:]))
        if s.dec_mlp_keys:
            feat = torch.cat([post_stoch.reshape(*post_deter.shape[:-1], -1), post_deter], -1)
            pre = "decoder._mlp.mlp.layers." + s.dec_mlp_name
            x = feat
            for i in range(s.dec_mlp_layers):
                x = F.silu(rms(F.linear(x, P[f"{pre}_linear{i}.weight"], P[f"{pre}_linear{i}.bias"]), P[f"{pre}_norm{i}.weight"]))
            x = F.linear(x, P["decoder._mlp.last.weight"], P["decoder._mlp.last.bias"])
            for k, mode in zip(s.dec_mlp_keys, torch.split(x, s.dec_mlp_split, -1)):
                d = (mode.to(DT) - symlog(data[k])) ** 2.0  # SymlogDist(mse, sum), distributions.py:174-190
                d = torch.where(d < 1e-8, 0, d)
                out[k] = torch.mean(d.sum(list(range(d.dim()))[2:]))
        return out

    def cal_grad(self, data, initial, seed, row_offset=0, keep=None):
        """Dreamer._cal_grad (dreamer.py:453-671) with autocast disabled (fp32). Returns (post, losses, metrics)."""
        s, M, P = self.s, self.model, self.P
        Pd = {k: v.detach() for k, v in P.items()}
        c = s.cfg
        losses, metrics = {}, {}
        B, T = data["action"].shape[:2]
        embed = M.encode(data)
        post_stoch, post_deter, post_logit = M.observe(embed, data["action"], initial, data["is_first"], seed, row_offset)
        prior_logit = M.img_logit(post_deter)  # rssm.prior (dreamer.py:485); its sample is discarded
        kf = float(c.kl_free)
        rep = torch.clip(kl_cat(post_logit, prior_logit.detach()).sum(-1), min=kf)  # rssm.py:222-230
        dyn = torch.clip(kl_cat(post_logit.detach(), prior_logit).sum(-1), min=kf)
        losses["dyn"] = torch.mean(dyn)
        losses["rep"] = torch.mean(rep)
        feat = M.get_feat(post_stoch, post_deter)
        if s.rep_loss == "dreamer":
            losses.update(self.decode_losses(data, post_stoch, post_deter))
        elif s.rep_loss == "r2dreamer":  # dreamer.py:497-532
            x1 = F.linear(feat.reshape(B * T, -1), P["prj.w.weight"])
            aug = c.r2dreamer.aug
            if bool(aug.enabled):  # _augment_images + random_translate (dreamer.py:716-729,845-880)
                with torch.no_grad():
                    pad, same = int(aug.max_delta), bool(aug.same_across_time)
                    sh = torch.from_numpy(nz.aug_shifts(seed, B, row_offset, T, pad, same))  # (B, T, 2): (x, y)
                    aug_img = random_translate(data["image"], sh, pad, bool(aug.bilinear))
                    x2 = M.encode({**data, "image": aug_img}).reshape(B * T, -1)
            else:
                x2 = embed.reshape(B * T, -1).detach()
            x1n = (x1 - x1.mean(0)) / (x1.std(0) + 1e-8)
            x2n = (x2 - x2.mean(0)) / (x2.std(0) + 1e-8)
            cc = torch.mm(x1n.T, x2n) / (B * T)
            inv = (torch.diagonal(cc) - 1.0).pow(2).sum()
            off = ~torch.eye(x1.shape[-1], dtype=torch.bool)
            red = cc[off].pow(2).sum()
            losses["barlow"] = inv + float(c.r2dreamer.lambd) * red
        elif s.rep_loss == "infonce":  # dreamer.py:533-542
            x1 = F.linear(feat.reshape(B * T, -1), P["prj.w.weight"])
            x2 = embed.reshape(B * T, -1).detach()
            logits = torch.matmul(x1, x2.T)
            norm_logits = logits - torch.max(logits, 1)[0][:, None]
            labels = torch.arange(norm_logits.shape[0]).long()
            losses["infonce"] = F.cross_entropy(norm_logits, labels)
        elif s.rep_loss == "dreamerpro":  # dreamer.py:543-566: doubled augmented batch, EMA targets, Sinkhorn
            assert row_offset == 0, "DreamerPro's Sinkhorn normalises over the whole batch: whole batches only"
            aug = c.dreamer_pro.aug
            pad, same = int(aug.max_delta), bool(aug.same_across_time)
            with torch.no_grad():  # augment_data (dreamer.py:731-743): rows [0, B) and [B, 2B) get their own shifts
                data_aug = {k: torch.cat([v, v], 0) for k, v in data.items()}
                sh = torch.from_numpy(nz.aug_shifts(seed, 2 * B, 0, T, pad, same))
                data_aug["image"] = random_translate(data_aug["image"], sh, pad, bool(aug.bilinear))
                init_aug = (torch.cat([initial[0], initial[0]], 0), torch.cat([initial[1], initial[1]], 0))
                Pe = {k: P[ek] for k, ek in s.ema_names.items()}  # ema_proj (dreamer.py:745-750)
                ema = F.linear(M.encode(data_aug, Pe), Pe["obs_proj.weight"], Pe["obs_proj.bias"])
                ema = F.normalize(ema, p=2, dim=-1)
            embed_aug = M.encode(data_aug)
            ps_aug, pd_aug, _ = M.observe(embed_aug, data_aug["action"], init_aug, data_aug["is_first"], seed, 0,
                                          nz.STREAM_OBS_AUG)
            losses.update(self.proto_loss(ps_aug, pd_aug, embed_aug, ema))
        else:
            raise NotImplementedError(s.rep_loss)
        losses["rew"] = torch.mean(-twohot_log_prob(M.head_logits("reward", feat), M.rbins, data["reward"].to(DT)))
        cont = 1.0 - data["is_terminal"].to(DT)
        losses["con"] = torch.mean(-bernoulli_log_prob(M.head_logits("cont", feat), cont))
        metrics["dyn_entropy"] = torch.mean(cat_entropy(unimix_logits(prior_logit, s.unimix)).sum(-1))
        metrics["rep_entropy"] = torch.mean(cat_entropy(unimix_logits(post_logit, s.unimix)).sum(-1))

        # imagination (dreamer.py:578-636)
        start = (post_stoch.reshape(-1, s.S, s.K).detach(), post_deter.reshape(-1, s.D).detach())
        H1 = int(c.imag_horizon) + 1
        rec = {} if keep is not None else None
        imag_feat, imag_action = M.imagine(start, H1, seed, row_offset * T, rec)
        imag_feat, imag_action = imag_feat.detach(), imag_action.detach()
        imag_reward = twohot_mode(M.head_logits("reward", imag_feat, Pd), M.rbins)
        imag_cont = torch.sigmoid(M.head_logits("cont", imag_feat, Pd).to(DT))  # Bernoulli.mean
        imag_value = twohot_mode(M.head_logits("value", imag_feat, Pd), M.bins)
        imag_slow_value = twohot_mode(M.head_logits("slow_value", imag_feat, Pd), M.bins)
        disc = 1 - 1 / int(c.horizon)
        weight = torch.cumprod(imag_cont * disc, dim=1)
        last = torch.zeros_like(imag_cont)
        term = 1 - imag_cont
        ret = lambda_return(last, term, imag_reward, imag_value, imag_value, disc, float(c.lamb))
        ret_offset, ret_scale = return_ema(self.ema_vals, ret)
        adv = (ret - imag_value[:, :-1]) / ret_scale
        pl = M.head_logits("actor", imag_feat)
        if s.discrete:
            nl = unimix_logits(pl, float(s.actor_dist.unimix_ratio))
            logpi = onehot_log_prob(nl, imag_action)[:, :-1].unsqueeze(-1)
            entropy = cat_entropy(nl)[:, :-1].unsqueeze(-1)
        else:
            loc, scale = bounded_normal_params(pl, float(s.actor_dist.min_std), float(s.actor_dist.max_std))
            logpi = normal_log_prob(loc, scale, imag_action)[:, :-1].unsqueeze(-1)
            entropy = normal_entropy(scale)[:, :-1].unsqueeze(-1)
        losses["policy"] = torch.mean(weight[:, :-1].detach() * -(logpi * adv.detach() + float(c.act_entropy) * entropy))
        vl = M.head_logits("value", imag_feat)
        tar_padded = torch.cat([ret, 0 * ret[:, -1:]], 1)
        losses["value"] = torch.mean(weight[:, :-1].detach() * (
            -twohot_log_prob(vl, M.bins, tar_padded.detach())
            - twohot_log_prob(vl, M.bins, imag_slow_value.detach()))[:, :-1].unsqueeze(-1))
        ret_normed = (ret - ret_offset) / ret_scale
        metrics["ret"] = torch.mean(ret_normed)
        metrics["ret_005"] = self.ema_vals[0].clone()
        metrics["ret_095"] = self.ema_vals[1].clone()
        metrics["adv"] = torch.mean(adv)
        metrics["adv_std"] = torch.std(adv)
        metrics["con"] = torch.mean(imag_cont)
        metrics["rew"] = torch.mean(imag_reward)
        metrics["val"] = torch.mean(imag_value)
        metrics["tar"] = torch.mean(ret)
        metrics["slowval"] = torch.mean(imag_slow_value)
        metrics["weight"] = torch.mean(weight)
        metrics["action_entropy"] = torch.mean(entropy)
        metrics.update(tensorstats(imag_action, "action"))

        # replay value (dreamer.py:638-664)
        last, term, reward = data["is_last"].to(DT), data["is_terminal"].to(DT), data["reward"].to(DT)
        boot = ret[:, 0].reshape(B, T, 1)
        value = twohot_mode(M.head_logits("value", feat, Pd), M.bins)
        slow_value = twohot_mode(M.head_logits("slow_value", feat, Pd), M.bins)
        wgt = 1.0 - last
        rret = lambda_return(last, term, reward, value, boot, disc, float(c.lamb))
        ret_padded = torch.cat([rret, 0 * rret[:, -1:]], 1)
        vd = M.head_logits("value", feat)
        losses["repval"] = torch.mean(wgt[:, :-1] * (
            -twohot_log_prob(vd, M.bins, ret_padded.detach())
            - twohot_log_prob(vd, M.bins, slow_value.detach()))[:, :-1].unsqueeze(-1))
        metrics.update(tensorstats(rret, "ret_replay"))
        metrics.update(tensorstats(value, "value_replay"))
        metrics.update(tensorstats(slow_value, "slow_value_replay"))
        total = sum(v * self.loss_scales[k] for k, v in losses.items())
        total.backward()
        metrics.update({f"loss/{k}": v for k, v in losses.items()})
        metrics["opt/loss"] = total
        if keep is not None:
            keep.update(dict(embed=embed, post_logit=post_logit, prior_logit=prior_logit, imag_feat=imag_feat,
                             imag_action=imag_action, ret=ret, imag_value=imag_value, imag_reward=imag_reward,
                             imag_cont=imag_cont, rret=rret,
                             imag_actor_logit=torch.stack(rec["imag_actor_logit"], 1),
                             imag_prior_logit=torch.stack(rec["imag_prior_logit"], 1)))
        return (post_stoch, post_deter), losses, metrics

    @torch.no_grad()
    def agc_(self):  # clip_grad_agc_ foreach path, utils/optim/agc.py:15-53
        ps = [p for p in self.trainable() if p.grad is not None]
        gs = [p.grad for p in ps]
        pn = torch._foreach_norm(ps, ord=2)
        gn = torch._foreach_norm(gs, ord=2)
        upper = torch._foreach_mul(torch._foreach_maximum(pn, self.pmin), self.agc)
        scale = torch._foreach_reciprocal(torch._foreach_maximum(torch._foreach_div(gn, upper), 1.0))
        torch._foreach_mul_(gs, scale)

    @torch.no_grad()
    def laprop_step(self):  # LaProp.step, utils/optim/laprop.py:46-118 (amsgrad/centered off, wd 0)
        lr = self.lr()
        b1, b2 = self.betas
        for p in self.trainable():
            if p.grad is None:
                continue
            g = p.grad.data
            st = self.state.setdefault(id(p), None)
            if st is None:
                st = dict(step=0, exp_avg=torch.zeros_like(p.data), exp_avg_lr_1=0.0, exp_avg_lr_2=0.0,
                          exp_avg_sq=torch.zeros_like(p.data))
                self.state[id(p)] = st
            st["step"] += 1
            st["exp_avg_sq"].mul_(b2).addcmul_(g, g, value=1 - b2)
            st["exp_avg_lr_1"] = st["exp_avg_lr_1"] * b1 + (1 - b1) * lr
            st["exp_avg_lr_2"] = st["exp_avg_lr_2"] * b2 + (1 - b2)
            bc1 = st["exp_avg_lr_1"] / lr if lr != 0.0 else 1.0
            step_size = 1 / bc1
            denom = st["exp_avg_sq"].div(st["exp_avg_lr_2"]).sqrt_().add_(self.eps)
            st["exp_avg"].mul_(b1).add_(g / denom, alpha=(1 - b1) * lr)
            p.data.add_(st["exp_avg"], alpha=-step_size)

    def ema_update(self):  # Dreamer.ema_update (dreamer.py:752-762)
        dpc = self.s.cfg.dreamer_pro
        with torch.no_grad():
            self.P["_prototypes"].copy_(F.normalize(self.P["_prototypes"], p=2, dim=-1))
            if self.ema_updates % int(dpc.ema_update_every) == 0:
                mix = float(dpc.ema_update_fraction) if self.ema_updates > 0 else 1.0
                for k, ek in self.s.ema_names.items():
                    self.P[ek].copy_(mix * self.P[k].data + (1 - mix) * self.P[ek])
        self.ema_updates += 1

    def sinkhorn(self, scores):  # Dreamer.sinkhorn (dreamer.py:764-790): log-space Sinkhorn-Knopp over (K, N)
        dpc = self.s.cfg.dreamer_pro
        Kp = scores.shape[0]
        log_q = F.log_softmax(scores.reshape(-1) / float(dpc.sinkhorn_eps), dim=0).reshape(Kp, -1)
        N = log_q.shape[1]
        for _ in range(int(dpc.sinkhorn_iters)):
            log_q = log_q - torch.logsumexp(log_q, dim=1, keepdim=True) - math.log(Kp)
            log_q = log_q - torch.logsumexp(log_q, dim=0, keepdim=True) - math.log(N)
        return torch.exp(log_q + math.log(N)).reshape(scores.shape)

    def proto_loss(self, post_stoch, post_deter, embed, ema_proj):  # Dreamer.proto_loss (dreamer.py:792-843)
        P, dpc = self.P, self.s.cfg.dreamer_pro
        w, tau = int(dpc.warm_up), float(dpc.temperature)
        protos = F.normalize(P["_prototypes"], p=2, dim=-1)
        B2, T = embed.shape[:2]

        def scores(x):  # (B2, T, Pd) unit rows -> (K, B2, T - warm_up)
            return (x.reshape(B2 * T, -1) @ protos.t()).reshape(B2, T, -1).permute(2, 0, 1)[:, :, w:]

        obs = F.linear(embed, P["obs_proj.weight"], P["obs_proj.bias"])
        obs_norm = obs.norm(dim=-1)
        obs_logits = F.log_softmax(scores(F.normalize(obs, p=2, dim=-1)) / tau, dim=0)
        o1, o2 = obs_logits.chunk(2, dim=1)
        e1, e2 = scores(ema_proj).chunk(2, dim=1)
        with torch.no_grad():
            t1, t2 = self.sinkhorn(e1), self.sinkhorn(e2)
        targets = torch.cat([t1, t2], 1)
        feat = F.linear(torch.cat([post_stoch.reshape(B2, T, -1), post_deter], -1), P["feat_proj.weight"],
                        P["feat_proj.bias"])
        feat_norm = feat.norm(dim=-1)
        feat_logits = F.log_softmax(scores(F.normalize(feat, p=2, dim=-1)) / tau, dim=0)
        swav = -0.5 * (t2 * o1).sum(0).mean() - 0.5 * (t1 * o2).sum(0).mean()
        temp = -(targets * feat_logits).sum(0).mean()
        norm = ((obs_norm - 1) ** 2).mean() + ((feat_norm - 1) ** 2).mean()
        return {"swav": swav, "temp": temp, "norm": norm}

    def update(self, data, initial, seed, row_offset=0, keep=None):
        """Dreamer.update (dreamer.py:402-451) minus sampling/autocast/GradScaler (no-op scale 1 on CPU)."""
        self.update_slow_target()
        if self.s.rep_loss == "dreamerpro":
            self.ema_update()
        post, losses, metrics = self.cal_grad(data, initial, seed, row_offset, keep)
        if self.s.rep_loss == "dreamerpro" and self.ema_updates < int(self.s.cfg.dreamer_pro.freeze_prototypes_iters):
            self.P["_prototypes"].grad.zero_()  # dreamer.py:424-425
        self.agc_()
        self.laprop_step()
        self.opt_step += 1  # scheduler.step()
        for p in self.trainable():
            p.grad = None
        metrics["opt/lr"] = self.lr()
        return post, losses, metrics
