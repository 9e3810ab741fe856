"""Networks of the Dreamer hot path (reference: world_model/networks.py), MI355X-native.

Module trees and parameter names are identical to the reference, so `state_dict()` keys and shapes match a
reference `latest.pt` (train.py:126-130). Two parameters are stored in a kernel-friendly layout internally and
converted at (de)serialisation time:
  * BlockLinear.weight: reference (O/G, I/G, G) (networks.py:40) <-> internal (G, O/G, I/G) (K-contiguous per block);
  * conv weights: reference (Co, Ci, kh, kw) <-> internal (Co, kh, kw, Ci) (NHWC implicit GEMM).
All forward/backward compute goes through sdreamer.ops (HIP kernels).
"""
from __future__ import annotations

import math
import os
import re

import torch
from torch import nn

from . import kernels as K
from . import ops


def _trunc_normal_(w, fan_in, outscale=1.0):
    std = 1.1368 * math.sqrt(1.0 / fan_in)  # weight_init_ (tools.py:76-100), fan_type "in"
    with torch.no_grad():
        nn.init.trunc_normal_(w, mean=0.0, std=std, a=-2.0 * std, b=2.0 * std)
        if outscale != 1.0:
            w.mul_(outscale)


class Linear(nn.Module):
    def __init__(self, inp, out, bias=True, outscale=1.0):
        super().__init__()
        self.in_features, self.out_features = int(inp), int(out)
        self.weight = nn.Parameter(torch.empty(self.out_features, self.in_features))
        self.bias = nn.Parameter(torch.zeros(self.out_features)) if bias else None
        _trunc_normal_(self.weight.data, self.in_features, outscale)

    def forward(self, x):
        return ops.linear(x, self.weight, self.bias)


class RMSNorm(nn.Module):
    def __init__(self, dim, eps=1e-4):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(int(dim)))
        self.eps = eps


class Act(nn.Module):
    """SiLU placeholder (fused into the preceding RMSNorm kernel); keeps the reference's module indices."""

    def forward(self, x):  # pragma: no cover - never called on the fused path
        raise RuntimeError("fused")


class Lambda(nn.Module):
    def forward(self, x):  # pragma: no cover
        raise RuntimeError("fused")


class BlockLinear(nn.Module):
    """networks.py:24-56. Internal weight layout (G, O/G, I/G)."""

    def __init__(self, in_ch, out_ch, blocks, outscale=1.0):
        super().__init__()
        self.in_ch, self.out_ch, self.blocks = int(in_ch), int(out_ch), int(blocks)
        G = self.blocks
        w = torch.empty(self.out_ch // G, self.in_ch // G, G)
        _trunc_normal_(w, (self.in_ch // G) * G, outscale)  # torch fan_in of (O/G, I/G, G) = I/G * G
        self.weight = nn.Parameter(w.permute(2, 0, 1).contiguous())
        self.bias = nn.Parameter(torch.zeros(self.out_ch))

    def forward(self, x):
        return ops.block_linear(x, self.weight, self.bias)

    @staticmethod
    def weight_to_ref(t):  # internal (G, O/G, I/G) -> reference (O/G, I/G, G)
        return t.permute(1, 2, 0)

    @staticmethod
    def weight_from_ref(t):
        return t.permute(2, 0, 1)

    def _save_to_state_dict(self, destination, prefix, keep_vars):
        w = self.weight if keep_vars else self.weight.detach()
        destination[prefix + "weight"] = w.permute(1, 2, 0).contiguous()
        destination[prefix + "bias"] = self.bias if keep_vars else self.bias.detach()

    def _load_from_state_dict(self, state_dict, prefix, *args, **kwargs):
        key = prefix + "weight"
        if key in state_dict and tuple(state_dict[key].shape) == (self.out_ch // self.blocks, self.in_ch // self.blocks,
                                                                  self.blocks):
            state_dict[key] = state_dict[key].permute(2, 0, 1).contiguous()
        super()._load_from_state_dict(state_dict, prefix, *args, **kwargs)


class Conv2d(nn.Module):
    """Conv2dSamePad (networks.py:59-85), stride 1. Internal weight layout (Co, kh, kw, Ci)."""

    def __init__(self, ci, co, k):
        super().__init__()
        self.ci, self.co, self.k = int(ci), int(co), int(k)
        w = torch.empty(self.co, self.ci, self.k, self.k)
        _trunc_normal_(w, self.ci * self.k * self.k)
        self.weight = nn.Parameter(w.permute(0, 2, 3, 1).contiguous())
        self.bias = nn.Parameter(torch.zeros(self.co))

    @staticmethod
    def weight_to_ref(t):  # internal (Co, kh, kw, Ci) -> reference (Co, Ci, kh, kw)
        return t.permute(0, 3, 1, 2)

    @staticmethod
    def weight_from_ref(t):
        return t.permute(0, 2, 3, 1)

    def _save_to_state_dict(self, destination, prefix, keep_vars):
        w = self.weight if keep_vars else self.weight.detach()
        destination[prefix + "weight"] = w.permute(0, 3, 1, 2).contiguous()
        destination[prefix + "bias"] = self.bias if keep_vars else self.bias.detach()

    def _load_from_state_dict(self, state_dict, prefix, *args, **kwargs):
        key = prefix + "weight"
        if key in state_dict and tuple(state_dict[key].shape) == (self.co, self.ci, self.k, self.k):
            state_dict[key] = state_dict[key].permute(0, 2, 3, 1).contiguous()
        super()._load_from_state_dict(state_dict, prefix, *args, **kwargs)


class MLP(nn.Module):
    """networks.py:313-336: [Linear -> RMSNorm -> SiLU] x layers (symlog inputs optional)."""

    def __init__(self, config, inp_dim):
        super().__init__()
        self._symlog_inputs = bool(config.symlog_inputs)
        self.layers = nn.Sequential()
        self.n = int(config.layers)
        for i in range(self.n):
            self.layers.add_module(f"{config.name}_linear{i}", Linear(inp_dim, config.units))
            self.layers.add_module(f"{config.name}_norm{i}", RMSNorm(config.units))
            self.layers.add_module(f"{config.name}_act{i}", Act())
            inp_dim = int(config.units)
        self.out_dim = int(config.units)
        self._mods = [(self.layers[3 * i], self.layers[3 * i + 1]) for i in range(self.n)]

    def forward(self, x, fast=False):
        if self._symlog_inputs:
            x = K.symlog(x.contiguous())
        for lin, norm in self._mods:
            x = ops.rms_silu(ops.linear(x, lin.weight, lin.bias, fast), norm.weight)
        return x

    def forward_from_first(self, x, h0, fast=False):
        """forward whose first linear output h0 = x . W0^T + b0 is given (ops.LinearPreFn: the backward still
        produces W0 / b0's gradients from x)."""
        (lin, norm), rest = self._mods[0], self._mods[1:]
        h = ops.rms_silu(ops.linear_pre(h0, x, lin.weight, lin.bias), norm.weight)
        for lin, norm in rest:
            h = ops.rms_silu(ops.linear(h, lin.weight, lin.bias, fast), norm.weight)
        return h

    @torch.no_grad()
    def forward_nograd(self, x, fast=False):
        if self._symlog_inputs:
            x = K.symlog(x.contiguous())
        for lin, norm in self._mods:
            x = K.rmsnorm_fwd(K.linear(x.reshape(-1, x.shape[-1]), lin.weight, lin.bias, fast=fast), norm.weight,
                              act=1)[0]
        return x


class MLPHead(nn.Module):
    """networks.py:339-377. Returns raw logits; distribution math lives in the callers (dreamer.py)."""

    def __init__(self, config, inp_dim):
        super().__init__()
        self.mlp = MLP(config, inp_dim)
        self.dist_name = str(config.dist.name)
        self.dist_cfg = config.dist
        shape = tuple(int(s) for s in config.shape)
        out = {"bounded_normal": 2 * shape[0], "onehot": shape[0], "multi_onehot": sum(shape)}.get(self.dist_name, shape[0])
        outscale = float(config.outscale) if config.outscale is not None else 1.0
        self.last = Linear(self.mlp.out_dim, out, outscale=outscale)

    def forward(self, x, fast=False):
        """fast: split-bf16 contractions (imagined trajectories; see ops.LinearFn)."""
        return ops.linear(self.mlp(x, fast), self.last.weight, self.last.bias, fast)

    def forward_from_first(self, x, h0, fast=False):
        """logits given the first layer's pre-norm output h0 (same rows as x), with gradients for every layer."""
        if self.mlp._symlog_inputs:
            return self.forward(x, fast)
        return ops.linear(self.mlp.forward_from_first(x, h0, fast), self.last.weight, self.last.bias, fast)

    def logits_rest(self, h, fast=False):
        """logits given the first layer's normalised, activated output h (ops.PairFirstFn)"""
        for lin, norm in self.mlp._mods[1:]:
            h = ops.rms_silu(ops.linear(h, lin.weight, lin.bias, fast), norm.weight)
        return ops.linear(h, self.last.weight, self.last.bias, fast)

    @torch.no_grad()
    def logits_nograd(self, x, fast=False):
        h = self.mlp.forward_nograd(x.reshape(-1, x.shape[-1]), fast)
        return K.linear(h, self.last.weight, self.last.bias, fast=fast)

    @torch.no_grad()
    def logits_from_first(self, h0, fast=False):
        """logits given the first layer's pre-norm output h0 = x . W0^T + b0 (see heads_nograd)."""
        (_, norm0), rest = self.mlp._mods[0], self.mlp._mods[1:]
        h = K.rmsnorm_fwd(h0, norm0.weight, act=1)[0]
        for lin, norm in rest:
            h = K.rmsnorm_fwd(K.linear(h, lin.weight, lin.bias, fast=fast), norm.weight, act=1)[0]
        return K.linear(h, self.last.weight, self.last.bias, fast=fast)


def pair_forward_from_first(ha, hb, x, h0a, h0b, fast=False):
    """Logits of two MLPHeads on the same detached rows x whose first linear outputs h0a / h0b are given; their first
    layers' backward is one joint weight-gradient GEMM (ops.PairFirstFn). None when the heads do not qualify."""
    if ha.mlp._symlog_inputs or hb.mlp._symlog_inputs or ha.mlp.n < 1 or hb.mlp.n < 1:
        return None
    (la, na), (lb, nb) = ha.mlp._mods[0], hb.mlp._mods[0]
    if la.bias is None or lb.bias is None or la.weight.shape[1] != lb.weight.shape[1]:
        return None
    ya, yb = ops.PairFirstFn.apply(h0a, h0b, x, la.weight, la.bias, na.weight, lb.weight, lb.bias, nb.weight)
    return ha.logits_rest(ya, fast), hb.logits_rest(yb, fast)


FUSED_HEADS = os.environ.get("SDREAMER_FUSED_HEADS", "1") != "0"


@torch.no_grad()
def heads_nograd(heads, x, fast=False, firsts_out=None):
    """Frozen logits of several MLPHeads on the same input rows x (M, F). The four first layers run as ONE batched
    launch (A = x broadcast over the heads: read once per row tile on one XCD, gemm3's tile order); with `fast` the
    rest of every head is fused too (_heads_rest_fused: each later layer applies the previous layer's RMSNorm + SiLU
    while staging its input, so no normalised tensor is written). Falls back to per-head forwards when the first
    layers differ in shape or use symlog. firsts_out (a list): receives the (n, M, U) first-layer outputs."""
    firsts = [h.mlp._mods[0][0] for h in heads]
    shape = tuple(firsts[0].weight.shape)
    if any(h.mlp._symlog_inputs or h.mlp.n < 1 for h in heads) or any(tuple(f.weight.shape) != shape for f in firsts):
        return [h.logits_nograd(x, fast) for h in heads]
    x = x.reshape(-1, x.shape[-1])
    M, n, U = x.shape[0], len(heads), shape[0]
    h0 = torch.empty(n, M, U, dtype=torch.float32, device=x.device)
    if fast and FUSED_HEADS and U % 64 == 0:
        p0 = torch.empty(n, U // 64, M, dtype=torch.float32, device=x.device)
        # per-entry weights: the heads' parameters are read in place (no stacked copies)
        if K.mlp_layer(x.expand(n, M, x.shape[1]), [f.weight for f in firsts], h0, bias=[f.bias for f in firsts],
                       part_out=p0):
            out = _heads_rest_fused(heads, h0, p0)
            if out is not None:
                if firsts_out is not None:
                    firsts_out.append(h0)
                return out
    w = torch.stack([f.weight for f in firsts])  # (n, U, F)
    b = torch.stack([f.bias for f in firsts])  # (n, U)
    K.gemm(x.expand(n, M, x.shape[1]), w.transpose(1, 2), h0, bias=b, fast=fast)
    if firsts_out is not None:
        firsts_out.append(h0)
    return [h.logits_from_first(h0[i], fast) for i, h in enumerate(heads)]


@torch.no_grad()
def _heads_rest_fused(heads, h0, p0):
    """Layers 1.. and the output layer of every head after the batched first layer, each a sd_gemm_bf16x3_mlp launch
    batched over the heads that share it: heads with the same depth run their hidden layers together (their
    activations are consecutive slices of one buffer), and the output layer of a depth group is one launch as wide as
    the group's widest head (the continue head's single logit rides with the reward head's 255; per-entry weight rows,
    so nothing is stacked or zero-padded). Returns None when a shape falls outside the fused kernel."""
    n, M, U = h0.shape
    dev = h0.device
    depth = [h.mlp.n for h in heads]
    bufs, parts = {0: (list(range(n)), h0, p0)}, {}
    for layer in range(1, max(depth)):
        idx = [i for i in range(n) if depth[i] > layer]
        prev_idx, prev_h, prev_p = bufs[layer - 1]
        pos = [prev_idx.index(i) for i in idx]
        if pos != list(range(pos[0], pos[0] + len(pos))):
            return None
        sl = slice(pos[0], pos[0] + len(pos))
        w = [heads[i].mlp._mods[layer][0].weight for i in idx]
        b = [heads[i].mlp._mods[layer][0].bias for i in idx]
        nw = [heads[i].mlp._mods[layer - 1][1].weight for i in idx]
        h = torch.empty(len(idx), M, U, dtype=torch.float32, device=dev)
        pt = torch.empty(len(idx), U // 64, M, dtype=torch.float32, device=dev)
        if not K.mlp_layer(prev_h[sl], w, h, bias=b, norm_w=nw, part_in=prev_p[sl], part_out=pt):
            return None
        bufs[layer] = (idx, h, pt)
    out = [None] * n
    for dep in sorted(set(depth)):
        idx = [i for i in range(n) if depth[i] == dep]
        src_idx, src_h, src_p = bufs[dep - 1]
        pos = [src_idx.index(i) for i in idx]
        if pos != list(range(pos[0], pos[0] + len(pos))):
            return None
        sl = slice(pos[0], pos[0] + len(pos))
        no = max(heads[i].last.weight.shape[0] for i in idx)
        no_p = max(no, 64)  # the launch's width; a narrower head's columns past its rows come out 0
        w = [heads[i].last.weight for i in idx]
        b = [heads[i].last.bias for i in idx]
        nw = [heads[i].mlp._mods[dep - 1][1].weight for i in idx]
        lg = torch.empty(len(idx), M, no_p, dtype=torch.float32, device=dev)
        if not K.mlp_layer(src_h[sl], w, lg, bias=b, norm_w=nw, part_in=src_p[sl]):
            return None
        for j, i in enumerate(idx):
            r = heads[i].last.weight.shape[0]
            out[i] = lg[j] if r == no_p else lg[j, :, :r]
    return out


class ConvEncoder(nn.Module):
    """networks.py:192-234. Input NHWC float in [0, 1] (B*T, 64, 64, 3); output (B*T, C*h*w) in NCHW flatten order."""

    def __init__(self, config, input_shape):
        super().__init__()
        h, w, ch = input_shape
        self.depths = tuple(int(config.depth) * int(m) for m in list(config.mults))
        self.k = int(config.kernel_size)
        if not bool(config.norm):
            raise NotImplementedError("norm=False encoder")
        layers = []
        inp = ch
        for d in self.depths:
            layers += [Conv2d(inp, d, self.k), Lambda(), RMSNorm(d), Act()]
            inp = d
            h, w = h // 2, w // 2
        self.layers = nn.Sequential(*layers)
        self.out_dim = self.depths[-1] * h * w

    def dgrad_weights(self):
        """conv weights whose input gradient the backward computes (every stage but the first)"""
        return [self.layers[4 * i].weight for i in range(1, len(self.depths))]

    def forward(self, obs, split=None):
        """split (a list): the first stage's output is continued as a detached leaf and (output, leaf) appended, so
        the backward runs as two calls (stages 2.. down to the leaf, then the first stage)."""
        x = obs
        n = len(self.depths)
        for i in range(n):
            conv, norm = self.layers[4 * i], self.layers[4 * i + 2]
            x = ops.ConvPoolNormFn.apply(x, conv.weight, conv.bias, norm.weight, i == n - 1)
            if i == 0 and n > 1 and split is not None and x.requires_grad:
                leaf = x.detach().requires_grad_(True)
                split.append((x, leaf))
                x = leaf
        return x


class MultiEncoder(nn.Module):
    """networks.py:99-141."""

    def __init__(self, config, shapes):
        super().__init__()
        excluded = ("is_first", "is_last", "is_terminal", "reward")
        shapes = {k: v for k, v in shapes.items() if k not in excluded and not k.startswith("log_")}
        self.cnn_shapes = {k: v for k, v in shapes.items() if len(v) == 3 and re.match(config.cnn_keys, k)}
        self.mlp_shapes = {k: v for k, v in shapes.items() if len(v) in (1, 2) and re.match(config.mlp_keys, k)}
        self.out_dim = 0
        encs = []
        self.kinds = []
        if self.cnn_shapes:
            ch = sum(v[-1] for v in self.cnn_shapes.values())
            shp = tuple(self.cnn_shapes.values())[0][:2] + (ch,)
            encs.append(ConvEncoder(config.cnn, shp))
            self.kinds.append("cnn")
            self.out_dim += encs[-1].out_dim
        if self.mlp_shapes:
            encs.append(MLP(config.mlp, sum(sum(v) for v in self.mlp_shapes.values())))
            self.kinds.append("mlp")
            self.out_dim += encs[-1].out_dim
        if not encs:
            raise NotImplementedError
        self.encoders = nn.ModuleList(encs)

    def dgrad_weights(self):
        return [w for kind, enc in zip(self.kinds, self.encoders) if kind == "cnn" for w in enc.dgrad_weights()]

    def forward(self, obs, split=None):
        """obs: dict of (B, T, *); images already float in [0, 1] (after preprocess). Returns (B, T, E).
        split: see ConvEncoder.forward."""
        outs = []
        for kind, enc in zip(self.kinds, self.encoders):
            if kind == "cnn":
                pre = obs.get("__enc_image")  # formed by Dreamer.preprocess(enc_input=True) from the uint8 bytes
                img = pre if pre is not None else (
                    torch.cat([obs[k] for k in self.cnn_shapes], -1) if len(self.cnn_shapes) > 1
                    else obs[next(iter(self.cnn_shapes))])
                BT = img.shape[:-3]
                x = img.reshape(-1, *img.shape[-3:])
                if pre is not None:
                    pass
                elif x.shape[-1] % 4:  # obs - 0.5 (networks.py:224), zero-padded to a float4 channel multiple
                    x = K.pad_channels(x.contiguous(), (x.shape[-1] + 3) // 4 * 4, 0.5)
                else:
                    x = x - 0.5  # ConvEncoder.forward, networks.py:224
                outs.append(enc(x.contiguous(), split).reshape(*BT, -1))
            else:
                x = torch.cat([obs[k] for k in self.mlp_shapes], -1)
                outs.append(enc(x))
        return outs[0] if len(outs) == 1 else torch.cat(outs, -1)


class ConvDecoder(nn.Module):
    """networks.py:237-310 (NHWC internally; output (..., H, W, C) like the reference)."""

    def __init__(self, config, deter, flat_stoch, shape=(3, 64, 64)):
        super().__init__()
        self._shape = shape
        self.depths = tuple(int(config.depth) * int(m) for m in list(config.mults))
        factor = 2 ** len(self.depths)
        minres = [int(x // factor) for x in shape[1:]]
        self.min_shape = (*minres, self.depths[-1])
        self.bspace = int(config.bspace)
        self.k = int(config.kernel_size)
        self.units = int(config.units)
        u, g = math.prod(self.min_shape), self.bspace
        self.sp0 = BlockLinear(deter, u, g)
        self.sp1 = nn.Sequential(Linear(flat_stoch, 2 * self.units), RMSNorm(2 * self.units), Act())
        self.sp2 = Linear(2 * self.units, u)
        self.sp_norm = nn.Sequential(RMSNorm(self.depths[-1]), Act())
        layers = []
        inp = self.depths[-1]
        for d in reversed(self.depths[:-1]):
            layers += [Lambda(), Conv2d(inp, d, self.k), RMSNorm(d), Act()]
            inp = d
        layers += [Lambda(), Conv2d(inp, shape[0], self.k)]
        self.layers = nn.Sequential(*layers)
        H, W, C = self.min_shape
        G = self.bspace
        # sp0 output column (g, y, x, c') -> channels-last (y, x, g*C/G + c')  (networks.py:290-292)
        idx = torch.arange(u).view(G, H, W, C // G).permute(1, 2, 0, 3).reshape(-1)
        self.register_buffer("_perm", idx, persistent=False)

    def forward(self, stoch, deter):
        BT = deter.shape[:-1]
        x0 = deter.reshape(-1, deter.shape[-1])
        x1 = stoch.reshape(x0.shape[0], -1)
        H, W, C = self.min_shape
        x0 = ops.block_linear(x0, self.sp0.weight, self.sp0.bias)
        x0 = x0.index_select(1, self._perm).view(-1, H, W, C)
        x1 = ops.rms_silu(ops.linear(x1, self.sp1[0].weight, self.sp1[0].bias), self.sp1[1].weight)
        x1 = ops.linear(x1, self.sp2.weight, self.sp2.bias).view(-1, H, W, C)
        x = ops.rms_silu(x0 + x1, self.sp_norm[0].weight)
        n = (len(self.layers) - 2) // 4
        for i in range(n):
            conv, norm = self.layers[4 * i + 1], self.layers[4 * i + 2]
            x = ops.UpConvFn.apply(x, conv.weight, conv.bias)
            x = ops.rms_silu(x, norm.weight)
        last = self.layers[4 * n + 1]
        x = ops.UpConvFn.apply(x, last.weight, last.bias)
        x = torch.sigmoid(x)
        return x.reshape(*BT, *x.shape[1:])


class MultiDecoder(nn.Module):
    """networks.py:144-189."""

    def __init__(self, config, deter, flat_stoch, shapes):
        super().__init__()
        excluded = ("is_first", "is_last", "is_terminal")
        shapes = {k: v for k, v in shapes.items() if k not in excluded}
        self.cnn_shapes = {k: v for k, v in shapes.items() if len(v) == 3 and re.match(config.cnn_keys, k)}
        self.mlp_shapes = {k: v for k, v in shapes.items() if len(v) in (1, 2) and re.match(config.mlp_keys, k)}
        self.all_keys = list(self.mlp_shapes.keys()) + list(self.cnn_shapes.keys())
        if self.cnn_shapes:
            some = list(self.cnn_shapes.values())[0]
            shape = (sum(x[-1] for x in self.cnn_shapes.values()),) + tuple(some[:-1])
            self._cnn = ConvDecoder(config.cnn, deter, flat_stoch, shape)
        if self.mlp_shapes:
            config.mlp.shape = (sum(sum(x) for x in self.mlp_shapes.values()),)
            self._mlp = MLPHead(config.mlp, deter + flat_stoch)
            self.mlp_dist = str(config.mlp_dist.name)
        self.cnn_dist = str(config.cnn_dist.name)

    def forward(self, stoch, deter):
        """Returns {key: mode tensor} (the distributions' parameters)."""
        out = {}
        if self.cnn_shapes:
            x = self._cnn(stoch, deter)
            for key, o in zip(self.cnn_shapes, torch.split(x, [v[-1] for v in self.cnn_shapes.values()], -1)):
                out[key] = o
        if self.mlp_shapes:
            feat = torch.cat([stoch.reshape(*deter.shape[:-1], -1), deter], -1)
            x = self._mlp(feat)
            for key, o in zip(self.mlp_shapes, torch.split(x, [v[0] for v in self.mlp_shapes.values()], -1)):
                out[key] = o
        return out


class Projector(nn.Module):
    """networks.py:380-387."""

    def __init__(self, in_ch1, in_ch2):
        super().__init__()
        self.w = Linear(in_ch1, in_ch2, bias=False)

    def forward(self, x):
        return ops.linear(x, self.w.weight, None)


class ReturnEMA(nn.Module):
    """networks.py:406-422; quantiles + EMA computed by one HIP kernel (no host sync)."""

    def __init__(self, device, alpha=1e-2):
        super().__init__()
        self.alpha = alpha
        self.range = (0.05, 0.95)
        self.register_buffer("ema_vals", torch.zeros(2, dtype=torch.float32, device=device))

    def __call__(self, x, offset_scale=None):
        os_ = torch.empty(2, dtype=torch.float32, device=x.device) if offset_scale is None else offset_scale
        K.return_ema(x.detach().reshape(-1), self.ema_vals, os_, alpha=self.alpha, q0=self.range[0], q1=self.range[1])
        return os_[0], os_[1]
