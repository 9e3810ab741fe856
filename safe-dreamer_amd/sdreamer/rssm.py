"""RSSM (reference: world_model/rssm.py), MI355X-native.

Same module tree / parameter names as the reference (`_deter_net._dyn_in{0,1,2}`, `_dyn_hid`, `_dyn_gru`, `_obs_net`,
`_img_net`), same public methods (`initial`, `observe`, `obs_step`, `img_step`, `prior`, `imagine_with_action`,
`get_feat`, `get_dist`-equivalents, `kl_loss`). Compute:

* `observe` is ONE autograd function (ObserveScan). Forward runs the L-step posterior scan; everything that does not
  depend on the recurrence is hoisted out of the loop and done as one (L*B)-row GEMM: the action branch
  (_dyn_in2 and its RMSNorm), the embed half of obs_net_0, and — in the backward — every weight gradient
  (sum over steps of dy_t^T x_t == one GEMM over the time-major (L*B) activations). The serial part of the
  backward only propagates data gradients (weights streamed once per step).
* `dyn_hid` is split into its block-diagonal deter part (a G-batched GEMM) and the part shared by all blocks
  ([x0, x1, x2] @ W_shared, rssm.py:52-58), so the (M, G*(D/G+3U)) concatenation is never materialised.
* imagination (Dreamer._imagine) is forward-only and runs on the kernels directly (no autograd graph).
"""
from __future__ import annotations

import ctypes
import os

import torch
from torch import nn

from . import _native as nat
from . import kernels as K
from . import ops
from .networks import Act, BlockLinear, Lambda, Linear, RMSNorm

STREAM_OBS, STREAM_IMG, STREAM_ACT, STREAM_POLICY, STREAM_POLICY_ACT = 1, 2, 3, 4, 5  # oracle/noise.py
STREAM_OBS_AUG = 7  # DreamerPro's augmented-view posterior scan
# the fused scan (csrc/scan.hip) is the default; SDREAMER_FUSED_SCAN=0 selects the per-op HIP kernels (tests compare)
FUSED_SCAN = os.environ.get("SDREAMER_FUSED_SCAN", "1") != "0"
# debugging aid: fill the fused backward's scratch tensors with NaN so any element read before it is written shows
_POISON = os.environ.get("SDREAMER_DEBUG_POISON", "0") != "0"
# rows per workgroup tile of the fused scan (csrc/scan.hip row_tile): every B rows run as ceil(B / tile) tiles in the
# same launches; 0 = the 16-row MFMA tile
SCAN_ROW_TILE = int(os.environ.get("SDREAMER_SCAN_ROWTILE", "0"))
# per direction (forward / backward launches), overriding SCAN_ROW_TILE when set
SCAN_ROW_TILE_FWD = int(os.environ.get("SDREAMER_SCAN_ROWTILE_FWD", "-1"))
SCAN_ROW_TILE_BWD = int(os.environ.get("SDREAMER_SCAN_ROWTILE_BWD", "-1"))
SCAN_KSD = int(os.environ.get("SDREAMER_SCAN_KSD", "8"))
SCAN_TRACE = None  # uint64 device tensor: per-launch / per-workgroup phase timestamps (tools/scan_trace.py)


def _fused_scan_ok(rssm, B):
    """Shapes csrc/scan.hip is instantiated for (every BASELINE config); others take the per-op HIP kernels."""
    D, U, G, SK, Kd = rssm._deter, rssm._hidden, rssm._blocks, rssm.flat_stoch, rssm._discrete
    if not FUSED_SCAN or B > 4096 or G > 8 or D % G or D > 4096:
        return False
    return U == 256 and D // G in (256, 512) and SK in (512, 1024) and Kd in (16, 32, 64) and D % Kd == 0 and \
        D % 64 == 0


def _scan_desc(rssm, P, B, T, seed, row_offset, rt, x2, eproj, work, stream_id=STREAM_OBS, bwd=False):
    d = nat.ScanDesc()
    D, U, SK, Kd, G = rssm._deter, rssm._hidden, rssm.flat_stoch, rssm._discrete, rssm._blocks
    d.B, d.T, d.D, d.U, d.SK, d.Kd, d.G = B, T, D, U, SK, Kd, G
    # K splits of the D-wide / SK-wide step GEMMs (slabs summed by the consumer): 8 D-wide slabs = 2 x the k_slab
    # workgroups of 4, each staging half the weight and deter bytes
    d.ks_d, d.ks_s = (SCAN_KSD if D % (16 * SCAN_KSD) == 0 else 4), 2
    side = SCAN_ROW_TILE_BWD if bwd else SCAN_ROW_TILE_FWD
    d.row_tile = side if side >= 0 else SCAN_ROW_TILE
    if SCAN_TRACE is not None:  # measurement aid (tools/scan_trace.py, a -DSD_SCAN_TRACE build of the library)
        d.trace = SCAN_TRACE.data_ptr()
    d.eps, d.unimix = K.EPS, rssm._unimix_ratio
    sh, sp = K.seed_args(seed)
    d.seed, d.seed_ptr, d.stream_id, d.group_offset = sh, sp, int(stream_id), int(row_offset) * rssm._stoch
    for k in ("W0", "b0", "n0", "W1", "b1", "n1", "Wh", "bh", "nh", "Wg", "bg", "Wl", "bl"):
        setattr(d, k, P[k].data_ptr())
    d.no = P["no"].data_ptr()
    d.reset, d.x2, d.eproj = rt.data_ptr(), x2.data_ptr(), eproj.data_ptr()
    d.reset_bm = 1  # the fused scan (this descriptor's only user) reads the batch-major (B, T) flags in place
    d.work = K.p(work)
    return d


def _scan_work(d):
    n = nat.fns["sd_rssm_scan_work_floats"](ctypes.addressof(d))
    if n < 0:
        raise nat.NativeError(f"sd_rssm_scan_work_floats failed with status {n}")
    return n


class Deter(nn.Module):
    """rssm.py:10-75 (parameters only; the step is computed by RSSM._deter_fwd / ObserveScan)."""

    def __init__(self, deter, stoch, act_dim, hidden, blocks, dynlayers, act="SiLU"):
        super().__init__()
        self.blocks = int(blocks)
        self.dynlayers = int(dynlayers)
        if self.dynlayers != 1:
            raise NotImplementedError("dyn_layers != 1 (base.yaml:266 uses 1)")
        self._dyn_in0 = nn.Sequential(Linear(deter, hidden), RMSNorm(hidden), Act())
        self._dyn_in1 = nn.Sequential(Linear(stoch, hidden), RMSNorm(hidden), Act())
        self._dyn_in2 = nn.Sequential(Linear(act_dim, hidden), RMSNorm(hidden), Act())
        self._dyn_hid = nn.Sequential()
        in_ch = (3 * hidden + deter // self.blocks) * self.blocks
        self._dyn_hid.add_module("dyn_hid_0", BlockLinear(in_ch, deter, self.blocks))
        self._dyn_hid.add_module("norm_0", RMSNorm(deter))
        self._dyn_hid.add_module("act_0", Act())
        self._dyn_gru = BlockLinear(deter, 3 * deter, self.blocks)


class RSSM(nn.Module):
    """rssm.py:78-230."""

    def __init__(self, config, embed_size, act_dim):
        super().__init__()
        self._stoch = int(config.stoch)
        self._deter = int(config.deter)
        self._hidden = int(config.hidden)
        self._discrete = int(config.discrete)
        self._unimix_ratio = float(config.unimix_ratio)
        self._bwd_tr = None  # scan_bwd_weights() computed ahead of the scan backward (Dreamer._ph_wm), or None
        self._bwd_extra = None  # (d_stoch2, d_deter2): second posterior-gradient summands for the next backward
        self._initial = str(config.initial)
        self._device = torch.device(config.device)
        self._act_dim = int(act_dim)
        self._obs_layers = int(config.obs_layers)
        self._img_layers = int(config.img_layers)
        self._blocks = int(config.blocks)
        if self._obs_layers != 1:
            raise NotImplementedError("obs_layers != 1 (base.yaml:264 uses 1)")
        self.flat_stoch = self._stoch * self._discrete
        self.feat_size = self.flat_stoch + self._deter
        self.embed_size = int(embed_size)
        self._deter_net = Deter(self._deter, self.flat_stoch, act_dim, self._hidden, self._blocks, config.dyn_layers)
        self._obs_net = nn.Sequential()
        self._obs_net.add_module("obs_net_0", Linear(self._deter + embed_size, self._hidden))
        self._obs_net.add_module("obs_net_n_0", RMSNorm(self._hidden))
        self._obs_net.add_module("obs_net_a_0", Act())
        self._obs_net.add_module("obs_net_logit", Linear(self._hidden, self.flat_stoch))
        self._obs_net.add_module("obs_net_lambda", Lambda())
        self._img_net = nn.Sequential()
        inp = self._deter
        for i in range(self._img_layers):
            self._img_net.add_module(f"img_net_{i}", Linear(inp, self._hidden))
            self._img_net.add_module(f"img_net_n_{i}", RMSNorm(self._hidden))
            self._img_net.add_module(f"img_net_a_{i}", Act())
            inp = self._hidden
        self._img_net.add_module("img_net_logit", Linear(inp, self.flat_stoch))
        self._img_net.add_module("img_net_lambda", Lambda())

    # ------------------------------------------------------------------ parameter views
    def _p(self):
        dn = self._deter_net
        D, G = self._deter, self._blocks
        Dg = D // G
        wh = dn._dyn_hid.dyn_hid_0.weight  # (G, Dg, Dg + 3U)
        Ig = wh.shape[2]
        return dict(
            W0=dn._dyn_in0[0].weight, b0=dn._dyn_in0[0].bias, n0=dn._dyn_in0[1].weight,
            W1=dn._dyn_in1[0].weight, b1=dn._dyn_in1[0].bias, n1=dn._dyn_in1[1].weight,
            W2=dn._dyn_in2[0].weight, b2=dn._dyn_in2[0].bias, n2=dn._dyn_in2[1].weight,
            Wh=wh, bh=dn._dyn_hid.dyn_hid_0.bias, nh=dn._dyn_hid.norm_0.weight,
            Wsh=wh.view(D, Ig)[:, Dg:], Wbd=wh[:, :, :Dg],
            Wg=dn._dyn_gru.weight, bg=dn._dyn_gru.bias,
            Wo=self._obs_net.obs_net_0.weight, bo=self._obs_net.obs_net_0.bias, no=self._obs_net.obs_net_n_0.weight,
            Wl=self._obs_net.obs_net_logit.weight, bl=self._obs_net.obs_net_logit.bias,
        )

    def scan_bwd_weights(self):
        """The transposed weight layouts sd_rssm_scan_bwd reads (W^T of the scan's contractions). Dreamer computes
        them on the main stream while it waits for the imagined returns, so the seven transposes are off the way
        from the head losses to the encoder gradient; the weights do not change until the optimizer step."""
        P = self._p()
        D = self._deter
        srcs = dict(W0T=P["W0"], W1T=P["W1"], WshT=P["Wsh"], WbdT=P["Wbd"], WgT=P["Wg"], WoDT=P["Wo"][:, :D],
                    WlT=P["Wl"])
        out, ents = {}, []
        for name, w in srcs.items():  # all seven transposes in one sd_layout_copies_run launch
            w3 = w if w.dim() == 3 else w.unsqueeze(0)
            nb, rows, cols = w3.shape
            if w3.stride(2) != 1:
                raise ValueError(f"{name}: rows must be contiguous")
            out[name] = torch.empty(nb, cols, rows, dtype=w.dtype, device=w.device)
            ents.append((w3, out[name], nb, rows, cols, w3.stride(0), w3.stride(1), cols, 0))
            if w.dim() == 2:
                out[name] = out[name][0]
        K.layout_copies(ents)
        return out

    def _img_mods(self):
        return [(self._img_net[3 * i], self._img_net[3 * i + 1]) for i in range(self._img_layers)], self._img_net.img_net_logit

    # ------------------------------------------------------------------ reference API
    def initial(self, batch_size):  # rssm.py:133-138 (always zeros; config.initial is unused there too)
        deter = torch.zeros(batch_size, self._deter, dtype=torch.float32, device=self._device)
        stoch = torch.zeros(batch_size, self._stoch, self._discrete, dtype=torch.float32, device=self._device)
        return stoch, deter

    def takes_extra_grads(self, B):
        """observe() on B rows is one ObserveScan, so its backward can take _bwd_extra"""
        return True

    def get_feat(self, stoch, deter):  # rssm.py:211-217
        return torch.cat([stoch.reshape(*stoch.shape[:-2], self.flat_stoch), deter], -1)

    def observe(self, embed, action, initial, reset, seed=0, row_offset=0, stream_id=STREAM_OBS):
        """rssm.py:140-156. embed (B,T,E), action (B,T,A), initial ((B,S,K),(B,D)), reset (B,T[,1]) bool.
        `seed`/`row_offset`/`stream_id` select the counter-based posterior noise (oracle/noise.py)."""
        B, T = action.shape[:2]
        r = reset.reshape(B, T)
        r = r.view(torch.uint8) if r.dtype == torch.bool and r.is_contiguous() else r.to(torch.uint8)  # no copy
        stoch0, deter0 = initial
        s0 = stoch0.reshape(B, -1)
        # rows are independent sequences: B > 16 runs as row tiles side by side inside every scan launch
        return ObserveScan.apply(embed, action, r, s0.contiguous(), deter0.contiguous(), self, seed, int(row_offset),
                                 stream_id)

    @torch.no_grad()
    def obs_step(self, stoch, deter, prev_action, embed, reset, seed=0, step=0, row_offset=0,
                 stream_id=STREAM_POLICY):
        """rssm.py:158-178 (no-grad form used by Dreamer.act)."""
        B = prev_action.shape[0]
        m = reset.reshape(B).to(torch.uint8).contiguous()
        s_in = K.mask_rows(stoch.reshape(B, -1).contiguous(), m)
        h_in = K.mask_rows(deter.contiguous(), m)
        a_in = K.action_norm(K.mask_rows(prev_action.contiguous(), m))
        deter = self._deter_fwd(s_in, h_in, a_in)
        P = self._p()
        D = self._deter
        op = K.linear(embed.contiguous(), P["Wo"][:, D:], P["bo"])
        K.gemm(deter, P["Wo"][:, :D].t(), op, beta=1.0)
        o, _ = K.rmsnorm_fwd(op, P["no"])
        logit = K.linear(o, P["Wl"], P["bl"])
        st = K.onehot_sample(logit, self._discrete, self._unimix_ratio, seed, stream_id, step, row_offset * self._stoch)
        S, Kd = self._stoch, self._discrete
        return st.view(B, S, Kd), deter, logit.view(B, S, Kd)

    @torch.no_grad()
    def img_step(self, stoch, deter, prev_action, seed=0, step=0, row_offset=0, stream_id=STREAM_IMG):
        """rssm.py:180-187."""
        M = prev_action.shape[0]
        a_in = K.action_norm(prev_action.contiguous())
        deter = self._deter_fwd(stoch.reshape(M, -1).contiguous(), deter.contiguous(), a_in)
        stoch, _ = self._prior_nograd(deter, seed, step, row_offset, stream_id)
        return stoch, deter

    def prior(self, deter):
        """rssm.py:189-195: logits of the prior with autograd (the reference's discarded sample is skipped)."""
        mods, last = self._img_mods()
        x = deter
        for lin, norm in mods:
            x = ops.rms_silu(ops.linear(x, lin.weight, lin.bias), norm.weight)
        x = ops.linear(x, last.weight, last.bias)
        return x.reshape(*x.shape[:-1], self._stoch, self._discrete)

    @torch.no_grad()
    def imagine_with_action(self, stoch, deter, actions, seed=0, row_offset=0):  # rssm.py:197-209
        T = actions.shape[1]
        stochs, deters = [], []
        for i in range(T):
            stoch, deter = self.img_step(stoch, deter, actions[:, i], seed=seed, step=i, row_offset=row_offset)
            stochs.append(stoch)
            deters.append(deter)
        return torch.stack(stochs, 1), torch.stack(deters, 1)

    def kl_loss(self, post_logit, prior_logit, free):  # rssm.py:222-230 (returns dyn, rep)
        S, Kd = self._stoch, self._discrete
        shp = post_logit.shape[:-2]
        dyn, rep = ops.KLFn.apply(post_logit.reshape(-1, S * Kd), prior_logit.reshape(-1, S * Kd), float(free), S, Kd)
        return dyn.view(shp), rep.view(shp)

    @torch.no_grad()
    def entropy(self, logit):
        """sum_S entropy of the unimix categorical (metrics dyn_entropy/rep_entropy, dreamer.py:575-576)."""
        S, Kd = self._stoch, self._discrete
        return self.entropy_terms(logit).view(-1, S).sum(-1)

    @torch.no_grad()
    def entropy_terms(self, logit):
        """per-categorical entropies (rows * S): the metric mean_rows sum_S is S * their mean (a K.Stat scale, no
        sum launch)"""
        Kd = self._discrete
        return K.onehot_entropy(logit.detach().reshape(-1, Kd).contiguous(), Kd, self._unimix_ratio)

    # ------------------------------------------------------------------ fused no-grad pieces
    @torch.no_grad()
    def _deter_fwd(self, s_in, h_in, a_n, x2=None):
        """Deter.forward (rssm.py:36-75) on masked/normalised inputs (M rows)."""
        P = self._p()
        M = h_in.shape[0]
        D, G, U = self._deter, self._blocks, self._hidden
        Dg = D // G
        xcat = torch.empty(M, 3 * U, dtype=torch.float32, device=h_in.device)
        K.rmsnorm_fwd(K.linear(h_in, P["W0"], P["b0"]), P["n0"], y=xcat[:, :U])
        K.rmsnorm_fwd(K.linear(s_in, P["W1"], P["b1"]), P["n1"], y=xcat[:, U:2 * U])
        if x2 is None:
            K.rmsnorm_fwd(K.linear(a_n, P["W2"], P["b2"]), P["n2"], y=xcat[:, 2 * U:])
        else:
            xcat[:, 2 * U:] = x2
        hp = K.mm(xcat, P["Wsh"].t(), bias=P["bh"])
        K.gemm(h_in.view(M, G, Dg).permute(1, 0, 2), P["Wbd"].transpose(1, 2), hp.view(M, G, Dg).permute(1, 0, 2),
               beta=1.0)
        h, _ = K.rmsnorm_fwd(hp, P["nh"])
        gates = torch.empty(M, 3 * D, dtype=torch.float32, device=h_in.device)
        K.gemm(h.view(M, G, Dg).permute(1, 0, 2), P["Wg"].transpose(1, 2), gates.view(M, G, 3 * Dg).permute(1, 0, 2),
               bias=P["bg"].view(G, 3 * Dg))
        return K.gru_fwd(gates, h_in, G)

    @torch.no_grad()
    def _prior_logits_nograd(self, deter):
        mods, last = self._img_mods()
        x = deter
        for lin, norm in mods:
            x = K.rmsnorm_fwd(K.linear(x, lin.weight, lin.bias), norm.weight)[0]
        return K.linear(x, last.weight, last.bias)

    @torch.no_grad()
    def _prior_nograd(self, deter, seed, step, row_offset, stream_id=STREAM_IMG):
        logit = self._prior_logits_nograd(deter)
        st = K.onehot_sample(logit, self._discrete, self._unimix_ratio, seed, stream_id, step, row_offset * self._stoch)
        return st, logit


SCAN_KEEP = None  # bench.py sets a dict: the next fused observe scan's descriptor and buffers are kept in it


class ObserveScan(torch.autograd.Function):
    """RSSM.observe (rssm.py:140-156) forward + BPTT backward on HIP kernels. Saved activations are time-major."""

    @staticmethod
    def forward(ctx, embed, action, reset, stoch0, deter0, rssm, seed, row_offset, stream_id=STREAM_OBS):
        P = rssm._p()
        B, T, A = action.shape
        E = embed.shape[-1]
        S, Kd, D, U, G = rssm._stoch, rssm._discrete, rssm._deter, rssm._hidden, rssm._blocks
        SK, Dg = S * Kd, D // G
        dev = embed.device
        f32 = torch.float32
        M = T * B
        fused = _fused_scan_ok(rssm, B)
        # reset flags: the fused scan reads the batch's (B, T) bytes in place (sd_rssm_scan.reset_bm); the per-op
        # path walks time-major rows
        rt = reset.contiguous() if fused else reset.t().contiguous()
        # ---- hoisted, recurrence-free work over all T*B rows. Fused scan: on the batch-major rows b*T + t, read by
        # the scan in place (bm_inputs); per-op path: time-major rows. The (M, E) embedding is never transposed
        # (emb_t: batch-major rows, see _wgrads).
        emb_t = embed.detach().reshape(M, E)
        if fused:
            a_n = K.action_norm(K.mask_rows(action.reshape(M, A).contiguous(), reset.reshape(M).contiguous()))
            eproj = K.linear(emb_t, P["Wo"][:, D:], P["bo"])
        else:
            act_t = action.transpose(0, 1).reshape(M, A).contiguous()
            a_n = K.action_norm(K.mask_rows(act_t, rt.reshape(M)))
            eproj = K.linear(emb_t, P["Wo"][:, D:], P["bo"]).view(B, T, U).transpose(0, 1).reshape(M, U).contiguous()
        x2p = K.linear(a_n, P["W2"], P["b2"])
        x2, r2 = K.rmsnorm_fwd(x2p, P["n2"])
        # ---- per-step buffers (time-major)
        s_in = torch.empty(T, B, SK, dtype=f32, device=dev)
        h_in = torch.empty(T, B, D, dtype=f32, device=dev)
        x0p = torch.empty(T, B, U, dtype=f32, device=dev)
        x1p = torch.empty(T, B, U, dtype=f32, device=dev)
        r0 = torch.empty(T, B, dtype=f32, device=dev)
        r1 = torch.empty(T, B, dtype=f32, device=dev)
        xcat = torch.empty(T, B, 3 * U, dtype=f32, device=dev)
        hp = torch.empty(T, B, D, dtype=f32, device=dev)
        hh = torch.empty(T, B, D, dtype=f32, device=dev)
        rh = torch.empty(T, B, dtype=f32, device=dev)
        gates = torch.empty(T, B, 3 * D, dtype=f32, device=dev)
        deter = torch.empty(T, B, D, dtype=f32, device=dev)
        op = eproj.view(T, B, U)  # obs_net_0 pre-norm accumulates the deter half in place
        oo = torch.empty(T, B, U, dtype=f32, device=dev)
        ro = torch.empty(T, B, dtype=f32, device=dev)
        logit = torch.empty(T, B, SK, dtype=f32, device=dev)
        if fused:
            # the posterior outputs written batch-major by the scan itself (the time-major deter / logit stay the
            # backward's saved activations); obs_net_0's deter half read in place from the full weight
            post = (torch.empty(B, T, S, Kd, dtype=f32, device=dev), torch.empty(B, T, D, dtype=f32, device=dev),
                    torch.empty(B, T, S, Kd, dtype=f32, device=dev))
            Wo = P["Wo"]
            d = _scan_desc(rssm, P, B, T, seed, row_offset, rt, x2, eproj, None, stream_id)
            d.bm_inputs, d.ld_wod = 1, Wo.stride(0)
            work = torch.empty(_scan_work(d), dtype=f32, device=dev)
            d.work, d.WoD = work.data_ptr(), Wo.data_ptr()
            d.stoch0, d.deter0 = stoch0.data_ptr(), deter0.data_ptr()
            op = torch.empty(T, B, U, dtype=f32, device=dev)  # eproj stays the (embed half + bias) input
            for k, v in (("s_in", s_in), ("h_in", h_in), ("x0p", x0p), ("x1p", x1p), ("r0", r0), ("r1", r1),
                         ("xcat", xcat), ("hp", hp), ("hh", hh), ("rh", rh), ("gates", gates), ("deter", deter),
                         ("op", op), ("oo", oo), ("ro", ro), ("logit", logit), ("post_stoch", post[0]),
                         ("post_deter", post[1]), ("post_logit", post[2])):
                setattr(d, k, v.data_ptr())
            d.stoch = None
            nat.call("sd_rssm_scan_fwd", ctypes.addressof(d), K.stream())
            if SCAN_KEEP is not None:  # measurement aid (bench.py): the descriptor and every buffer it points to
                SCAN_KEEP.update(desc=d, work=work, WoD=Wo, bufs=(s_in, h_in, x0p, x1p, r0, r1, xcat, hp, hh, rh,
                                                                  gates, deter, op, oo, ro, logit, x2, eproj, rt,
                                                                  stoch0, deter0) + post, T=T, B=B)
        else:
            stoch = torch.empty(T, B, SK, dtype=f32, device=dev)
            xcat[:, :, 2 * U:] = x2.view(T, B, U)
        prev_s, prev_h = stoch0, deter0
        for t in (range(0) if fused else range(T)):
            m = rt[t]
            K.mask_rows(prev_s, m, out=s_in[t])
            K.mask_rows(prev_h, m, out=h_in[t])
            K.linear(h_in[t], P["W0"], P["b0"], out=x0p[t])
            K.rmsnorm_fwd(x0p[t], P["n0"], y=xcat[t, :, :U], rstd=r0[t])
            K.linear(s_in[t], P["W1"], P["b1"], out=x1p[t])
            K.rmsnorm_fwd(x1p[t], P["n1"], y=xcat[t, :, U:2 * U], rstd=r1[t])
            K.gemm(xcat[t], P["Wsh"].t(), hp[t], bias=P["bh"])
            K.gemm(h_in[t].view(B, G, Dg).permute(1, 0, 2), P["Wbd"].transpose(1, 2),
                   hp[t].view(B, G, Dg).permute(1, 0, 2), beta=1.0)
            K.rmsnorm_fwd(hp[t], P["nh"], y=hh[t], rstd=rh[t])
            K.gemm(hh[t].view(B, G, Dg).permute(1, 0, 2), P["Wg"].transpose(1, 2),
                   gates[t].view(B, G, 3 * Dg).permute(1, 0, 2), bias=P["bg"].view(G, 3 * Dg))
            K.gru_fwd(gates[t], h_in[t], G, out=deter[t])
            K.gemm(deter[t], P["Wo"][:, :D].t(), op[t], beta=1.0)
            K.rmsnorm_fwd(op[t], P["no"], y=oo[t], rstd=ro[t])
            K.linear(oo[t], P["Wl"], P["bl"], out=logit[t])
            K.onehot_sample(logit[t], Kd, rssm._unimix_ratio, seed, stream_id, t, row_offset * S, out=stoch[t])
            prev_s, prev_h = stoch[t], deter[t]
        ctx.save_for_backward(rt, a_n, x2p, r2, emb_t, s_in, h_in, x0p, x1p, r0, r1, xcat, hp, hh, rh, gates, deter,
                              op, oo, ro, logit)
        ctx.rssm, ctx.seed, ctx.row_offset, ctx.stream_id = rssm, seed, row_offset, stream_id
        ctx.set_materialize_grads(False)  # a posterior output without a gradient reaches the backward as None
        ctx.dims = (B, T, A, E)
        ctx.fused = fused
        if fused:
            ctx.x2 = x2
            return post
        post_stoch = stoch.transpose(0, 1).reshape(B, T, S, Kd).contiguous()
        post_deter = deter.transpose(0, 1).contiguous()
        post_logit = logit.transpose(0, 1).reshape(B, T, S, Kd).contiguous()
        return post_stoch, post_deter, post_logit

    @staticmethod
    def backward(ctx, d_stoch, d_deter, d_logit):
        (rt, a_n, x2p, r2, emb_t, s_in, h_in, x0p, x1p, r0, r1, xcat, hp, hh, rh, gates, deter, op, oo, ro,
         logit) = ctx.saved_tensors
        rssm = ctx.rssm
        P = rssm._p()
        B, T, A, E = ctx.dims
        S, Kd, D, U, G = rssm._stoch, rssm._discrete, rssm._deter, rssm._hidden, rssm._blocks
        SK, Dg = S * Kd, D // G
        M = T * B
        dev = logit.device
        f32 = torch.float32

        def tm(x, width):
            if x is None:
                return torch.zeros(T, B, width, dtype=f32, device=dev)
            return x.reshape(B, T, width).transpose(0, 1).contiguous()

        gb = ops.grad_buf
        # second summands of the posterior gradient handed over by the caller (Dreamer._ph_scan_bwd: the replay-value
        # feat gradient's stoch / deter halves), summed where the scan reads them
        extra, rssm._bwd_extra = rssm._bwd_extra, None
        if ctx.fused:
            dl_all, d_op, d_gates, d_hp, d_x0p, d_x1p, norm_w = ObserveScan._bwd_fused(
                ctx, d_stoch, d_deter, d_logit, rt, s_in, h_in, x0p, x1p, r0, r1, hp, rh, gates, op, ro, logit, extra)
            return ObserveScan._wgrads(ctx, P, rt, a_n, x2p, r2, emb_t, s_in, h_in, xcat, hh, deter, oo, dl_all,
                                       d_op, d_gates, d_hp, d_x0p, d_x1p, None, norm_w)
        if extra is not None:
            d_stoch = extra[0].reshape(B, T, SK) + (0 if d_stoch is None else d_stoch.reshape(B, T, SK))
            d_deter = extra[1] + (0 if d_deter is None else d_deter)
        ds_out = tm(d_stoch, SK)
        dd_out = tm(d_deter, D)
        dl_all = tm(d_logit, SK)  # becomes d logit (incl. the straight-through sample gradient) in place
        d_op = torch.empty(T, B, U, dtype=f32, device=dev)
        d_gates = torch.empty(T, B, 3 * D, dtype=f32, device=dev)
        d_hp = torch.empty(T, B, D, dtype=f32, device=dev)
        d_x0p = torch.empty(T, B, U, dtype=f32, device=dev)
        d_x1p = torch.empty(T, B, U, dtype=f32, device=dev)
        d_x2 = torch.empty(T, B, U, dtype=f32, device=dev)
        carry_s = torch.zeros(B, SK, dtype=f32, device=dev)
        carry_h = torch.zeros(B, D, dtype=f32, device=dev)
        for t in reversed(range(T)):
            ds = ds_out[t] + carry_s
            K.onehot_sample_bwd(logit[t], ds, Kd, rssm._unimix_ratio, ctx.seed, ctx.stream_id, t, ctx.row_offset * S,
                                dlogits=dl_all[t], accumulate=True)
            d_o = K.mm(dl_all[t], P["Wl"])
            K.rmsnorm_bwd(op[t], P["no"], ro[t], d_o, dx=d_op[t], dw=gb(P["no"]))
            dh = dd_out[t] + carry_h
            K.gemm(d_op[t], P["Wo"][:, :D], dh, beta=1.0)
            d_hin = torch.empty(B, D, dtype=f32, device=dev)
            K.gru_bwd(gates[t], h_in[t], dh, G, dgates=d_gates[t], dh=d_hin)
            d_h = torch.empty(B, D, dtype=f32, device=dev)
            K.gemm(d_gates[t].view(B, G, 3 * Dg).permute(1, 0, 2), P["Wg"], d_h.view(B, G, Dg).permute(1, 0, 2))
            K.rmsnorm_bwd(hp[t], P["nh"], rh[t], d_h, dx=d_hp[t], dw=gb(P["nh"]))
            d_xcat = K.mm(d_hp[t], P["Wsh"])
            K.gemm(d_hp[t].view(B, G, Dg).permute(1, 0, 2), P["Wbd"], d_hin.view(B, G, Dg).permute(1, 0, 2), beta=1.0)
            d_x2[t] = d_xcat[:, 2 * U:]
            K.rmsnorm_bwd(x0p[t], P["n0"], r0[t], d_xcat[:, :U].contiguous(), dx=d_x0p[t], dw=gb(P["n0"]))
            K.gemm(d_x0p[t], P["W0"], d_hin, beta=1.0)
            K.rmsnorm_bwd(x1p[t], P["n1"], r1[t], d_xcat[:, U:2 * U].contiguous(), dx=d_x1p[t], dw=gb(P["n1"]))
            d_sin = K.mm(d_x1p[t], P["W1"])
            m = rt[t]
            carry_h = K.mask_rows(d_hin, m)
            carry_s = K.mask_rows(d_sin, m)
        return ObserveScan._wgrads(ctx, P, rt, a_n, x2p, r2, emb_t, s_in, h_in, xcat, hh, deter, oo, dl_all, d_op,
                                   d_gates, d_hp, d_x0p, d_x1p, d_x2)

    @staticmethod
    def _bwd_fused(ctx, d_stoch, d_deter, d_logit, rt, s_in, h_in, x0p, x1p, r0, r1, hp, rh, gates, op, ro, logit,
                   extra=None):
        """Serial part of the backward as sd_rssm_scan_bwd (6 fused launches per step) + the RMSNorm weight
        gradients of the four in-loop norms as (T*B)-row reductions."""
        rssm = ctx.rssm
        P = rssm._p()
        B, T, A, E = ctx.dims
        S, Kd, D, U, G = rssm._stoch, rssm._discrete, rssm._deter, rssm._hidden, rssm._blocks
        SK = S * Kd
        M = T * B
        dev = logit.device
        f32 = torch.float32

        def bm(x, width):  # the incoming gradients are read batch-major in place (bm_grads)
            return None if x is None else x.reshape(B, T, width).contiguous()

        ds_out, dd_out, dl_in = bm(d_stoch, SK), bm(d_deter, D), bm(d_logit, SK)
        e = lambda *shape: (torch.full(shape, float("nan"), dtype=f32, device=dev) if _POISON  # noqa: E731
                            else torch.empty(*shape, dtype=f32, device=dev))
        dl, d_o, d_op, d_x0p, d_x1p = e(T, B, SK), e(T, B, U), e(T, B, U), e(T, B, U), e(T, B, U)
        ctx.d_op_b = e(B, T, U)  # the batch-major copy k_dgru writes beside d_op (operand of the embed gradient)
        ctx.d_x2_b = e(B, T, U)  # the action branch's input gradient, batch-major (k_carry / k_dx01)
        d_gates, d_hh, d_hp, d_xcat = e(T, B, 3 * D), e(T, B, D), e(T, B, D), e(T, B, 3 * U)
        tr = rssm._bwd_tr if rssm._bwd_tr is not None else rssm.scan_bwd_weights()
        x2 = ctx.x2
        d = _scan_desc(rssm, P, B, T, ctx.seed, ctx.row_offset, rt, x2, x2, None, ctx.stream_id, bwd=True)
        work = e(_scan_work(d))
        d.work = work.data_ptr()
        for k, v in list(tr.items()) + [("s_in", s_in), ("h_in", h_in), ("x0p", x0p), ("x1p", x1p), ("r0", r0),
                                         ("r1", r1), ("hp", hp), ("rh", rh), ("gates", gates), ("op", op),
                                         ("ro", ro), ("logit", logit), ("dl", dl), ("d_o", d_o), ("d_op", d_op),
                                         ("d_gates", d_gates), ("d_hh", d_hh), ("d_hp", d_hp),
                                         ("d_xcat", d_xcat), ("d_x0p", d_x0p), ("d_x1p", d_x1p)]:
            setattr(d, k, v.data_ptr())
        d.d_stoch, d.d_deter, d.d_logit = K.p(ds_out), K.p(dd_out), K.p(dl_in)
        d.d_op_bm, d.d_x2_bm = ctx.d_op_b.data_ptr(), ctx.d_x2_b.data_ptr()
        d.bm_grads = 1
        if extra is not None:
            gs2, gd2 = extra
            # the kernels index row (b, t) as (b*T + t) * ld_g2: unit column stride, one row stride for both halves,
            # and the (B, T) rows evenly spaced; otherwise the explicit adds (the caller's former torch.add order)
            if gs2.stride(-1) == 1 and gd2.stride(-1) == 1 and gs2.stride(-2) == gd2.stride(-2) and \
                    gs2.stride(-3) == T * gs2.stride(-2) and gd2.stride(-3) == T * gd2.stride(-2):
                d.d_stoch2, d.d_deter2, d.ld_g2 = gs2.data_ptr(), gd2.data_ptr(), gs2.stride(-2)
            else:  # (not the benched path: DxSink's halves are strided views of one (B, T, F) buffer) both halves
                # copied into one (B, T, SK + D) buffer, whose two column blocks share a row stride; kept on ctx until
                # the backward's launches have run
                g2 = torch.cat([gs2.reshape(B, T, -1), gd2.reshape(B, T, -1)], -1)
                ctx.g2_hold = g2
                d.d_stoch2, d.d_deter2, d.ld_g2 = g2.data_ptr(), g2[..., SK:].data_ptr(), g2.stride(1)
        nat.call("sd_rssm_scan_bwd", ctypes.addressof(d), K.stream())
        gb = ops.grad_buf
        f = lambda x: x.reshape(M, -1)  # noqa: E731

        def norm_w():
            """the four in-loop norms' weight gradients and d_x2 (deferred with the weight-gradient GEMMs: nothing on
            the way to the encoder's gradient reads them)"""
            K.rmsnorm_bwd(f(op), P["no"], ro.reshape(M), f(d_o), dw=gb(P["no"]))
            K.rmsnorm_bwd(f(hp), P["nh"], rh.reshape(M), f(d_hh), dw=gb(P["nh"]))
            K.rmsnorm_bwd(f(x0p), P["n0"], r0.reshape(M), f(d_xcat)[:, :U], dw=gb(P["n0"]))  # column blocks in place
            K.rmsnorm_bwd(f(x1p), P["n1"], r1.reshape(M), f(d_xcat)[:, U:2 * U], dw=gb(P["n1"]))
            # the action branch ran on batch-major rows (ObserveScan.forward, fused path): k_carry / k_dx01 wrote
            # its gradient batch-major too (d_x2_bm)
            return ctx.d_x2_b

        norm_w.tensors = (op, hp, x0p, x1p, ro, rh, r0, r1, d_o, d_hh, d_xcat)
        return dl, d_op, d_gates, d_hp, d_x0p, d_x1p, norm_w

    @staticmethod
    def _wgrads(ctx, P, rt, a_n, x2p, r2, emb_t, s_in, h_in, xcat, hh, deter, oo, dl_all, d_op, d_gates, d_hp,
                d_x0p, d_x1p, d_x2, norm_w=None):
        """Deferred weight gradients: one GEMM (or column sum) over all T*B time-major rows each (split-bf16 GEMMs).
        norm_w (fused path): the in-loop norms' weight gradients, run first; returns d_x2."""
        rssm = ctx.rssm
        B, T, A, E = ctx.dims
        D, G = rssm._deter, rssm._blocks
        Dg = D // G
        M = T * B
        gb = ops.grad_buf
        f = lambda x: x.reshape(M, -1)  # noqa: E731
        # batch-major d_op (a (M, U) copy), so the embed gradient comes out in the encoder's (B, T, E) order directly
        d_op_b = getattr(ctx, "d_op_b", None)
        d_op_b = d_op.transpose(0, 1).reshape(M, -1).contiguous() if d_op_b is None else d_op_b.view(M, -1)
        d_emb = K.mm(d_op_b, P["Wo"][:, D:], fast=True)  # (M, E): the only output the encoder waits for

        def wgrads(d_x2=d_x2):
            if norm_w is not None:
                d_x2 = norm_w()
            K.wgrad(f(dl_all), f(oo), gb(P["Wl"]), gb(P["bl"]))  # weight + bias gradient, one launch
            gWo = gb(P["Wo"])
            K.wgrad(f(d_op), f(deter), gWo[:, :D], gb(P["bo"]))
            K.gemm(d_op_b.t(), emb_t, gWo[:, D:], beta=1.0, fast=True)  # both batch-major
            K.gemm(f(d_gates).view(M, G, 3 * Dg).permute(1, 2, 0), f(hh).view(M, G, Dg).permute(1, 0, 2),
                   gb(P["Wg"]), beta=1.0, fast=True)
            K.colsum(f(d_gates), gb(P["bg"]))
            gWh = gb(P["Wh"])
            Ig = gWh.shape[2]
            K.wgrad(f(d_hp), f(xcat), gWh.view(D, Ig)[:, Dg:], gb(P["bh"]))
            K.gemm(f(d_hp).view(M, G, Dg).permute(1, 2, 0), f(h_in).view(M, G, Dg).permute(1, 0, 2), gWh[:, :, :Dg],
                   beta=1.0, fast=True)
            K.wgrad(f(d_x0p), f(h_in), gb(P["W0"]), gb(P["b0"]))
            K.wgrad(f(d_x1p), f(s_in), gb(P["W1"]), gb(P["b1"]))
            d_x2p = K.rmsnorm_bwd(x2p, P["n2"], r2, f(d_x2), dw=gb(P["n2"]))
            K.wgrad(d_x2p, a_n, gb(P["W2"]), gb(P["b2"]))

        if ops._DEFER is not None:  # queued (ops.defer_wgrads): the caller runs them on another stream
            keep = (a_n, x2p, r2, emb_t, s_in, h_in, xcat, hh, deter, oo, dl_all, d_op, d_op_b, d_gates, d_hp, d_x0p,
                    d_x1p)
            keep += (d_x2,) if d_x2 is not None else norm_w.tensors
            ops._DEFER.append((wgrads, keep))
        else:
            wgrads()
        return d_emb.view(B, T, E), None, None, None, None, None, None, None, None
