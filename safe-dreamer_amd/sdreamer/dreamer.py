"""Dreamer agent (reference: world_model/dreamer.py), MI355X-native.

Public surface kept from the reference: `Dreamer(config.model, obs_space, act_space)`,
`.update(replay_buffer) -> metrics`, `._cal_grad`, `._imagine`, `._lambda_return`, `.act(obs, state, eval)`,
`.get_initial_state(B)`, `.preprocess`, `._named_params`, `state_dict()` with the reference's keys (including the
`_frozen_*` aliases), optimizer found at `._optimizer` / `._scheduler.optimizer`.

Differences by design (documented in DESIGN.md):
  * fp32 end to end (the reference's fp16 autocast + GradScaler are replaced by exact-f32 MFMA); `opt/grad_scale`=1;
  * sampling noise is counter-based (seed, stream, step, global row) instead of torch's global RNG, so results are
    reproducible across devices and identical under data-parallel sharding; `update()` draws seed = base + count;
  * imagination / heads are time-major internally; returned tensors use the reference layouts;
  * data parallel: `rank`/`world` row offsets for the noise, RCCL all-reduce of the flat gradient arena, global
    ReturnEMA quantiles (all-gather) and Barlow statistics (sdreamer/parallel.py).
"""
from __future__ import annotations

import contextlib
import copy
import ctypes
import math
import os
from collections import OrderedDict

import torch
import torch.distributed as dist
import torch.nn.functional as F
from torch import nn

from . import _native as nat
from . import kernels as K
from . import ops
from . import parallel
from .networks import (Linear, MLPHead, MultiDecoder, MultiEncoder, Projector, ReturnEMA, heads_nograd,
                       pair_forward_from_first)
from .optim import LaProp, WarmupSchedule
from .rssm import RSSM, STREAM_ACT, STREAM_IMG, STREAM_OBS_AUG, STREAM_POLICY, STREAM_POLICY_ACT

# SDREAMER_S2_AFTER_SCAN=1 (schedule knob): the actor/critic phase starts after the scan backward (beside the encoder
# backward) instead of right after the replay-value backward (beside the scan backward)
S2_AFTER_SCAN = os.environ.get("SDREAMER_S2_AFTER_SCAN", "0") == "1"
# graphed update, opt-in: the world-model heads' weight-gradient contractions leave phase M1 (which runs beside the
# imagination and slows it) for phase M2d on main after the encoder backward. Measured: the imagination got 0.27 ms
# faster but M2d (0.68 ms) outgrew the join slack it fills: 13.59 vs 13.34 ms per update, so off by default.
DEFER_WM = os.environ.get("SDREAMER_DEFER_WM", "0") == "1"
# graphed update: the first N queued encoder weight-gradient contractions (the last stages', queued first) run on main
# after the first stage's backward (phase M2d) instead of on the side stream (S4), which ends the update
S4_MAIN = int(os.environ.get("SDREAMER_S4_MAIN", "1"))  # measured: 0 -> 13.01, 1 -> 12.93, 2 -> 12.98 ms
# SDREAMER_FUSED_SAMPLE=0: replayed updates sample through Buffer.sample() + copies instead of sample_into (A/B knob)
FUSED_SAMPLE = os.environ.get("SDREAMER_FUSED_SAMPLE", "1") != "0"

# csrc/img.hip runs the whole imagination as 9 fused launches per step; SDREAMER_FUSED_IMAG=0 selects the per-op
# HIP kernels (tests compare the two)
FUSED_IMAG = os.environ.get("SDREAMER_FUSED_IMAG", "1") != "0"
# the policy / value losses start from first-layer outputs computed earlier in the update (the imagination's fp32
# actor layer 0, the imagined heads' batched value layer 0) instead of re-contracting the imagined feats;
# SDREAMER_REUSE_H0=0 recomputes them (A/B knob)
REUSE_H0 = os.environ.get("SDREAMER_REUSE_H0", "1") != "0"
# SDREAMER_PRIO=1 (schedule knob): graph-replayed updates run the critical chain on high-priority streams and the filler
# phases (M1, S2-S4) on normal-priority ones
STREAM_PRIO = os.environ.get("SDREAMER_PRIO", "0") == "1"
# SDREAMER_IMAG_NOISE=0: the imagined prior samples draw their Gumbel noise inside the sampler epilogue (per step)
# instead of from one sd_imagine_noise launch ahead of the rollout (same values; A/B knob)
IMAG_NOISE = os.environ.get("SDREAMER_IMAG_NOISE", "1") != "0"
# SDREAMER_FILL_CUS=first:count (schedule knob): the filler phases (M1 beside the imagination, S2-S4 beside the backward)
# replay on streams whose workgroups may run only on CUs [first, first + count) (sd_stream_create_cumask), so the
# latency-bound chain beside them keeps the other CUs to itself; the chain's own streams stay unmasked
FILL_CUS = os.environ.get("SDREAMER_FILL_CUS", "")
# SDREAMER_AC_DEFER=1 (schedule knob): the actor / value weight-gradient contractions of phase S2 (the imagined
# trajectories' large (H*N)-row GEMMs) are queued and run at the start of S3, beside the encoder backward, instead of
# beside the scan backward (M2a, the latency-bound chain S2 slows)
AC_DEFER = os.environ.get("SDREAMER_AC_DEFER", "0") == "1"
# the imagined actor's and value head's first-layer weight gradients as ONE split-bf16 GEMM over their joint dy: the
# 157 MB imagined-feature operand read once instead of twice (ops.PairFirstFn). 0 = one per head
PAIR_FIRST = os.environ.get("SDREAMER_PAIR_FIRST", "1") != "0"
# SDREAMER_SLOW_IN_S2=1: the imagined slow-critic head in the actor-critic phase S2 instead of with the other imagined
# heads in S1 (which end the path to the lambda-returns and the replay-value loss). Measured slower (10.87 -> 10.91 ms
# per update, profiles/r06f: the heads' batched first layer loses its fourth entry's reuse of the imagined features
# and S2 beside the scan backward grows), so off
SLOW_IN_S2 = os.environ.get("SDREAMER_SLOW_IN_S2", "0") == "1"
# KB of dynamic LDS every GEMM launch of the filler phases (M1, S2, S3, S4) reserves without using it (sd_set_lds_pad):
# fewer filler workgroups fit on a CU, leaving LDS for the latency-bound chain's workgroups beside them (0 = off)
FILL_LDS = int(os.environ.get("SDREAMER_FILL_LDS", "0"))
# S0: the imagination's noise and weight images (1), and also the scan backward's transposed and the encoder's flipped
# weights (2), as a side-stream phase beside the encoder forward instead of at the head of S1 (imagination) and inside
# M1. Measured neutral (profiles/r05v, r05w: the encoder forward slows by what S1 / M1 save; 3-round A/B 10.90 / 10.91 /
# 10.96 ms for 0 / 1 / 2): off by default
SIDE_PREP = int(os.environ.get("SDREAMER_SIDE_PREP", "0"))
# SDREAMER_SIDE_PREP_AT=scan: S0 forks off after the encoder forward, beside the posterior scan (a latency-bound chain
# of ~128-workgroup launches that leaves most CUs idle) instead of beside the compute-bound encoder: phase P gets a
# split point there (parallel.collective) whose host step records an event and queues S0 on the side stream
SIDE_PREP_AT = os.environ.get("SDREAMER_SIDE_PREP_AT", "enc")


def _symexp_bins(n, device):  # symexp_twohot bins, distributions.py:242-251
    if n % 2 == 1:
        half = torch.linspace(-20, 0, (n - 1) // 2 + 1, dtype=torch.float32)
        half = torch.sign(half) * torch.expm1(torch.abs(half))
        bins = torch.cat([half, -half[:-1].flip(0)], 0)
    else:
        half = torch.linspace(-20, 0, n // 2, dtype=torch.float32)
        half = torch.sign(half) * torch.expm1(torch.abs(half))
        bins = torch.cat([half, -half.flip(0)], 0)
    return bins.to(device)


def _tstats(t, prefix):  # tools.tensorstats (tools.py:275-281), resolved with the other metrics in one launch
    return K.tensorstats(t, prefix)



IMAG_TRACE = None  # uint64 device tensor: per-launch / per-workgroup phase timestamps of the fused imagination
_CUMASK = {}  # device -> the two CU-masked filler streams of SDREAMER_FILL_CUS (created once per process, never leaked
# per agent: tests and benches build several agents)


def _cumask_streams(device):
    key = str(device)
    if key not in _CUMASK:
        first, count = (int(v) for v in FILL_CUS.split(":"))
        mk = []
        for _ in range(2):
            h = ctypes.c_void_p()
            nat.call("sd_stream_create_cumask", first, count, ctypes.addressof(h))
            mk.append(torch.cuda.ExternalStream(h.value, device=device))
        _CUMASK[key] = tuple(mk)
    return _CUMASK[key]


class Dreamer(nn.Module):
    def __init__(self, config, obs_space, act_space, rank=0, world=1):
        super().__init__()
        self.device = torch.device(config.device)
        if self.device.type != "cuda":
            raise RuntimeError("sdreamer.Dreamer runs on a HIP device only (config.device must be cuda:N)")
        self.config = config
        self.act_entropy = float(config.act_entropy)
        self.kl_free = float(config.kl_free)
        self.imag_horizon = int(config.imag_horizon)
        self.horizon = int(config.horizon)
        self.lamb = float(config.lamb)
        self.return_ema = ReturnEMA(device=self.device)
        self.act_dim = act_space.n if hasattr(act_space, "n") else sum(act_space.shape)
        self.rep_loss = str(config.rep_loss)
        self.rank, self.world = int(rank), int(world)
        shapes = {k: tuple(v.shape) for k, v in obs_space.spaces.items()}
        if bool(config.use_multimodal_encoder):
            raise NotImplementedError("multimodal CLIP encoder is out of scope (SURVEY.md §2: OUT OF SCOPE)")
        self.encoder = MultiEncoder(config.encoder, shapes)
        self.embed_size = self.encoder.out_dim
        self.rssm = RSSM(config.rssm, self.embed_size, self.act_dim)
        self.reward = MLPHead(config.reward, self.rssm.feat_size)
        self.cont = MLPHead(config.cont, self.rssm.feat_size)
        config.actor.shape = (act_space.n,) if hasattr(act_space, "n") else tuple(map(int, act_space.shape))
        self.act_discrete = False
        if hasattr(act_space, "multi_discrete"):
            raise NotImplementedError("multi_discrete actions")
        elif hasattr(act_space, "discrete"):
            if "name" not in config.actor.dist:
                config.actor.dist = config.actor.dist.disc
            self.act_discrete = True
        elif "name" not in config.actor.dist:
            config.actor.dist = config.actor.dist.cont
        self.actor = MLPHead(config.actor, self.rssm.feat_size)
        self.value = MLPHead(config.critic, self.rssm.feat_size)
        self.slow_target_update = int(config.slow_target_update)
        self.slow_target_fraction = float(config.slow_target_fraction)
        self._slow_value = copy.deepcopy(self.value)
        for p in self._slow_value.parameters():
            p.requires_grad = False
        self._slow_value_updates = 0
        self._loss_scales = dict(config.loss_scales)
        # d total / d repval as a device scalar: the replay-value backward starts from it (no scaling kernels)
        self._repval_scale = torch.full((), float(self._loss_scales["repval"]), device=self.device)
        self._log_grads = bool(config.log_grads)
        modules = {"rssm": self.rssm, "actor": self.actor, "value": self.value, "reward": self.reward,
                   "cont": self.cont, "encoder": self.encoder}
        if self.rep_loss == "dreamer":
            self.decoder = MultiDecoder(config.decoder, self.rssm._deter, self.rssm.flat_stoch, shapes)
            recon = self._loss_scales.pop("recon")
            self._loss_scales.update({k: recon for k in self.decoder.all_keys})
            modules["decoder"] = self.decoder
        elif self.rep_loss in ("r2dreamer", "infonce"):
            self.prj = Projector(self.rssm.feat_size, self.embed_size)
            modules["projector"] = self.prj
            self.barlow_lambd = float(config.r2dreamer.lambd)
            aug = config.r2dreamer.aug
            # Barlow target from a translated view (dreamer.py:506-520): (pad, same_across_time) or None
            self.r2_aug = (int(aug.max_delta), bool(aug.same_across_time), bool(aug.get("bilinear", False))) if \
                (self.rep_loss == "r2dreamer" and bool(aug.enabled)) else None
        elif self.rep_loss == "dreamerpro":  # dreamer.py:131-162
            dpc = config.dreamer_pro
            self._pro = dict(warm_up=int(dpc.warm_up), tau=float(dpc.temperature), eps=float(dpc.sinkhorn_eps),
                             iters=int(dpc.sinkhorn_iters), every=int(dpc.ema_update_every),
                             frac=float(dpc.ema_update_fraction), freeze=int(dpc.freeze_prototypes_iters),
                             pad=int(dpc.aug.max_delta), same=bool(dpc.aug.same_across_time),
                             bilinear=bool(dpc.aug.get("bilinear", False)))
            self._prototypes = nn.Parameter(torch.randn(int(dpc.num_prototypes), int(dpc.proto_dim)))
            self.obs_proj = Linear(self.embed_size, int(dpc.proto_dim))
            self.feat_proj = Linear(self.rssm.feat_size, int(dpc.proto_dim))
            self._ema_encoder = copy.deepcopy(self.encoder)
            self._ema_obs_proj = copy.deepcopy(self.obs_proj)
            for prm in list(self._ema_encoder.parameters()) + list(self._ema_obs_proj.parameters()):
                prm.requires_grad = False
            self._ema_updates = 0
            modules.update({"prototypes": self._prototypes, "obs_proj": self.obs_proj, "feat_proj": self.feat_proj})
        else:
            raise NotImplementedError(f"rep_loss={self.rep_loss}")
        self._named_params = OrderedDict()
        for name, module in modules.items():
            if isinstance(module, nn.Parameter):
                self._named_params[name] = module
                continue
            for pn, prm in module.named_parameters():
                if prm.requires_grad:
                    self._named_params[f"{name}.{pn}"] = prm
        super().to(self.device)
        # parameters whose internal layout differs from the reference's (BlockLinear, Conv2d weights): how to view a
        # tensor of that parameter's shape (its gradient, its LaProp moments) in the reference layout and back
        packed = {}
        for name, module in modules.items():
            if isinstance(module, nn.Parameter):
                continue
            for mn, m in module.named_modules():
                if hasattr(m, "weight_to_ref"):
                    packed[f"{name}.{mn}.weight" if mn else f"{name}.weight"] = (m.weight_to_ref, m.weight_from_ref)
        self._ref_layouts = [packed.get(n) for n in self._named_params]
        self._optimizer = LaProp(self._named_params.values(), lr=float(config.lr),
                                 betas=(float(config.beta1), float(config.beta2)), eps=float(config.eps),
                                 agc=float(config.agc), pmin=float(config.pmin), warmup=int(config.warmup or 0),
                                 ref_layouts=self._ref_layouts, order=self._arena_order())
        self._scheduler = WarmupSchedule(self._optimizer)
        # slow critic arena mirrors the value head's slice of the parameter arena (one Polyak kernel)
        a = self._optimizer.arena
        vparams = [p for n, p in self._named_params.items() if n.startswith("value.")]
        pos = {id(p): i for i, p in enumerate(a.params)}
        idx = [pos[id(p)] for p in vparams]
        self._v_lo, self._v_hi = a.offsets[idx[0]], a.offsets[idx[-1]] + a.sizes[idx[-1]]
        self._slow_arena = a.data[self._v_lo:self._v_hi].clone()
        for p, sp in zip(vparams, self._slow_value.parameters()):
            j = pos[id(p)]
            o = a.offsets[j] - self._v_lo
            sp.data = self._slow_arena[o:o + a.sizes[j]].view(sp.shape)
        if self.rep_loss == "dreamerpro":  # EMA encoder / projection: arena-slice mirrors (one Polyak launch each)
            self._ema_mirrors = [self._mirror("encoder.", self._ema_encoder),
                                 self._mirror("obs_proj.", self._ema_obs_proj)]
            self._proto_gate = torch.ones(1, device=self.device)  # 0 while the prototypes are frozen
            # the fused optimizer step reads the prototype gradient times this gate (dreamer.py:424-425)
            self._optimizer.gate = (pos[id(self._prototypes)], self._proto_gate)
        self.rbins = _symexp_bins(int(config.reward.dist.bin_num), self.device)
        self.vbins = _symexp_bins(int(config.critic.dist.bin_num), self.device)
        self._updates = 0
        self.use_graphs = True
        # the actor-critic branch (imagination, policy/value/replay-value losses and their backward) depends only on the
        # detached posterior: it runs on this side stream concurrently with the world-model branch (see _cal_grad)
        self.use_side_stream = os.environ.get("SDREAMER_SIDE_STREAM", "1") != "0"
        # SDREAMER_MARKS=1: device timestamps at the phase boundaries of every update (kernels.Marks)
        self.marks = K.Marks(self.device) if os.environ.get("SDREAMER_MARKS", "0") != "0" else None
        self._side = torch.cuda.Stream(device=self.device)
        self._prio_streams = None  # (main, side, fill, side fill) of STREAM_PRIO, created at the first replay
        # device 1.0: the seed gradient of the world-model total (no fill launch per update); made here, outside any
        # capture, so its value never depends on which update first asks for it
        self._one = torch.ones((), dtype=torch.float32, device=self.device)
        self._comm = None  # data parallel: the gradient all-reduce stream (created on first use)
        self._buckets = self._grad_buckets()
        self._graph = None
        self._eager_updates = 0
        self._step_zeroes = False  # graph replays: the optimizer step zeroes the gradients (_update_graphed)
        self._grads_clean = False
        self._seed_base = int(getattr(config, "seed", 0) or 0) * 1_000_003 + 12345
        self.train()

    # ------------------------------------------------------------------ reference API
    def to(self, *args, **kwargs):  # dreamer.py:324-328 (frozen copies alias the live tensors by construction)
        dev = torch.device(args[0]) if args and isinstance(args[0], (str, torch.device)) else None
        if dev is not None and dev.type == "cuda" and (dev.index or 0) == (self.device.index or 0):
            return self
        return super().to(*args, **kwargs)

    def set_task_name(self, task_name):  # dreamer.py:235-240 (no-op without the multimodal encoder)
        pass

    def train(self, mode=True):
        super().train(mode)
        self._slow_value.train(False)
        return self

    def _update_slow_target(self):  # dreamer.py:242-249
        if self._slow_value_updates % self.slow_target_update == 0:
            self._polyak()
        self._slow_value_updates += 1

    def _polyak(self):
        K.polyak(self._optimizer.arena.data[self._v_lo:self._v_hi], self._slow_arena, self.slow_target_fraction)

    def _mirror(self, prefix, module):
        """A non-trainable copy of the contiguous arena slice holding `prefix`'s parameters; `module`'s parameters
        become views of it (DreamerPro's EMA encoder / obs projection)."""
        a = self._optimizer.arena
        pos = {id(p): i for i, p in enumerate(a.params)}
        idx = [pos[id(p)] for n, p in self._named_params.items() if n.startswith(prefix)]
        if idx != list(range(idx[0], idx[0] + len(idx))):
            raise RuntimeError(f"{prefix} parameters are not contiguous in the arena")
        lo, hi = a.offsets[idx[0]], a.offsets[idx[-1]] + a.sizes[idx[-1]]
        buf = a.data[lo:hi].clone()
        mps = list(module.parameters())
        if len(mps) != len(idx):
            raise RuntimeError(f"{prefix} mirror has {len(mps)} parameters for {len(idx)} arena slots")
        for j, mp in zip(idx, mps):
            o = a.offsets[j] - lo
            mp.data = buf[o:o + a.sizes[j]].view(mp.shape)
        return lo, hi, buf

    @torch.no_grad()
    def _ema_apply(self, mix):
        """dreamer.py:752-762 on device: unit prototypes, EMA encoder / projection <- mix * online + (1 - mix) * EMA."""
        pr = self._prototypes
        pr.copy_(pr / pr.norm(dim=-1, keepdim=True).clamp_min(1e-12))
        if mix is not None:
            a = self._optimizer.arena.data
            for lo, hi, buf in self._ema_mirrors:
                K.polyak(a[lo:hi], buf, mix)

    def ema_update(self):  # Dreamer.ema_update, dreamer.py:752-762
        c = self._pro
        self._ema_apply((c["frac"] if self._ema_updates > 0 else 1.0) if self._ema_updates % c["every"] == 0
                        else None)
        self._ema_updates += 1

    def _protos_frozen(self):  # dreamer.py:424-425 (checked after ema_update has counted this update)
        return self.rep_loss == "dreamerpro" and self._ema_updates < self._pro["freeze"]

    @torch.no_grad()
    def preprocess(self, data, enc_input=False):  # dreamer.py:709-713
        """enc_input: also form the ConvEncoder's input (image / 255 - 0.5, channel-padded) in the same launch
        ("__enc_image", read by MultiEncoder); the f32 image itself is then written only when a loss reads it
        (decoder, augmented views), else "image" stays the uint8 replay bytes."""
        if "image" in data and data["image"].dtype == torch.uint8:
            u8 = data["image"].contiguous()
            C = u8.shape[-1]
            if enc_input and C % 4 and self.encoder.cnn_shapes and list(self.encoder.cnn_shapes) == ["image"]:
                need = self.rep_loss in ("dreamer", "dreamerpro") or getattr(self, "r2_aug", None) is not None
                f, data["__enc_image"] = K.u8_image_inputs(u8, (C + 3) // 4 * 4, 0.5, need_f32=need)
                if f is not None:
                    data["image"] = f
            else:
                data["image"] = K.u8_to_f32(u8)
        return data

    @torch.no_grad()
    def get_initial_state(self, B):  # dreamer.py:359-363
        stoch, deter = self.rssm.initial(B)
        action = torch.zeros(B, self.act_dim, dtype=torch.float32, device=self.device)
        return {"stoch": stoch, "deter": deter, "prev_action": action}

    @torch.no_grad()
    def act(self, obs, state, eval=False, seed=None, step=0):
        """dreamer.py:330-357. obs: dict of (B, *) (image uint8), state: {stoch, deter, prev_action}."""
        p_obs = self.preprocess(dict(obs))
        embed = self.encoder({k: v.unsqueeze(1) for k, v in p_obs.items() if k in self.encoder.cnn_shapes
                              or k in self.encoder.mlp_shapes})[:, 0]
        B = embed.shape[0]
        seed = self._seed_base + 7 if seed is None else seed
        stoch, deter, _ = self.rssm.obs_step(state["stoch"], state["deter"], state["prev_action"], embed,
                                             obs["is_first"], seed=seed, step=step, stream_id=STREAM_POLICY)
        feat = self.rssm.get_feat(stoch, deter)
        logits = self.actor.logits_nograd(feat)
        if eval:
            if self.act_discrete:
                idx = logits.argmax(-1)  # argmax of unimix logits == argmax of raw logits
                action = torch.nn.functional.one_hot(idx, self.act_dim).float()
            else:
                action = torch.tanh(logits[:, : self.act_dim])  # Normal mean = tanh(mean) (dreamer act uses .mode)
        else:
            action = self._sample_action(logits, seed, step, 0, STREAM_POLICY_ACT)
        return action, {"stoch": stoch, "deter": deter, "prev_action": action}

    @torch.no_grad()
    def video_pred(self, data, initial, seed=0):
        """dreamer.py:366-400 (rep_loss == "dreamer" only): posterior over the first 5 steps, then open-loop
        imagination on the logged actions (RSSM.imagine_with_action, rssm.py:197-209), both decoded; returns
        cat([truth, model, (model - truth + 1) / 2], 2): (min(B, 6), T, 3H, W, C)."""
        if self.rep_loss != "dreamer":
            raise NotImplementedError("video_pred requires decoder and is only supported when rep_loss == 'dreamer'.")
        p = self.preprocess(dict(data))
        B = min(p["action"].shape[0], 6)
        embed = self.encoder(p)
        ps, pd, _ = self.rssm.observe(embed[:B, :5], p["action"][:B, :5].contiguous(),
                                      tuple(v[:B].contiguous() for v in initial), p["is_first"][:B, :5].contiguous(),
                                      seed=seed)
        recon = self.decoder(ps, pd)["image"][:B]
        if p["action"].shape[1] > 5:
            st, de = self.rssm.imagine_with_action(ps[:, -1].contiguous(), pd[:, -1].contiguous(),
                                                   p["action"][:B, 5:].contiguous(), seed=seed)
            model = torch.cat([recon[:, :5], self.decoder(st, de)["image"]], 1)
        else:  # sequences of <= 5 steps have no open-loop part (the reference's torch.stack would fail there)
            model = recon
        truth = p["image"][:B]
        error = (model - truth + 1.0) / 2.0
        return torch.cat([truth, model, error], 2)

    def policy_graph(self, B, obs_example, eval=False):
        """Dreamer.act for B environments as one replayed HIP graph (latency path).
        Returns policy(obs, state) -> (action, state): copies obs/state into the graph's static inputs, replays, and
        returns views of the graph's static outputs (valid until the next call). Call k samples exactly as
        act(obs, state, eval, seed=seed_base + k, step=0) does (the per-step seed lives on the device)."""
        dev = self.device
        s_obs = {k: torch.zeros_like(v, device=dev) for k, v in obs_example.items()}
        s_state = self.get_initial_state(B)
        seed_dev = torch.zeros(1, dtype=torch.int64, device=dev)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            act, st = self.act(s_obs, s_state, eval=eval, seed=seed_dev, step=0)
        counter = [0]
        base = self._seed_base + 7

        def policy(obs, state):
            for k, v in obs.items():
                s_obs[k].copy_(v)
            for k in ("stoch", "deter", "prev_action"):
                s_state[k].copy_(state[k])
            seed_dev.fill_(base + counter[0])
            counter[0] += 1
            g.replay()
            return act, st

        policy.graph, policy.counter = g, counter
        return policy

    def _sample_action(self, logits, seed, step, row_offset, stream_id):
        d = self.config.actor.dist
        if self.act_discrete:
            return K.onehot_sample(logits.contiguous(), self.act_dim, float(d.unimix_ratio), seed, stream_id, step,
                                   row_offset)
        out = torch.empty(logits.shape[0], self.act_dim, dtype=torch.float32, device=logits.device)
        sh, sp = K.seed_args(seed)
        K.nat.call("sd_bnormal_sample", K.p(logits.contiguous()), K.p(out), logits.shape[0], self.act_dim,
                   float(d.min_std), float(d.max_std), sh, stream_id, int(step), int(row_offset), sp, K.stream())
        return out

    # ------------------------------------------------------------------ update
    def update(self, replay_buffer):
        """dreamer.py:402-451."""
        if self._graph is not None and FUSED_SAMPLE and hasattr(replay_buffer, "sample_into") and \
                self.slow_target_update == 1:
            # replayed update: the replay slices are gathered straight into the graphs' input buffers (one launch)
            index = replay_buffer.sample_into(self._g_in, self._g_init)
            seed = self._seed_base + self._updates
            (stoch, deter), mets = self._update_graphed(None, None, seed, self._g_ro)
            replay_buffer.update(index, stoch.detach(), deter.detach())
            return mets
        data, index, initial = replay_buffer.sample()
        seed = self._seed_base + self._updates
        (stoch, deter), mets = self.update_batch(data, initial, seed)
        replay_buffer.update(index, stoch.detach(), deter.detach())
        return mets

    def update_batch(self, data, initial, seed, row_offset=None):
        """One optimisation step on a given batch. After two eager warm-up updates the update is captured into HIP
        graphs (set `use_graphs = False` to stay eager); multi-GPU runs split the graphs at the RCCL exchange steps
        (parallel.collective) and issue those eagerly between graph replays."""
        ro = self.rank * data["action"].shape[0] if row_offset is None else row_offset
        if self.use_graphs and self.slow_target_update == 1 and \
                (self.rep_loss != "dreamerpro" or self._pro["every"] == 1):
            if self._graph is not None or self._eager_updates >= 2:
                return self._update_graphed(data, initial, seed, ro)
        self._eager_updates += 1
        if self.marks is not None:
            self.marks.reset()
        p_data = self.preprocess(dict(data), enc_input=True)
        self._update_slow_target()
        if self.rep_loss == "dreamerpro":
            self.ema_update()
        self._optimizer.zero_grad()
        post, mets = self._cal_grad(p_data, initial, seed, ro)
        mets = K.resolve_metrics(mets)
        if self.rep_loss == "dreamerpro":
            self._proto_gate.fill_(0.0 if self._protos_frozen() else 1.0)
        if self.world > 1:
            parallel.allreduce_mean_(self._optimizer.arena.grad)
        self._optimizer.grad_scale = 1.0  # the eager all-reduce above already took the mean
        self._optimizer.step()
        self._mark("optimizer")
        self._scheduler.step()
        mets["opt/lr"] = self._scheduler.get_lr()[0]
        mets["opt/grad_scale"] = 1.0
        self._updates += 1
        return post, mets

    def _arena_order(self):
        """Physical order of the parameter arena: the named order, except that the actor's first linear weight closes
        the actor's block, so that it sits right before the value head's first linear weight (the value block's first
        tensor, kept contiguous for the slow critic's Polyak mirror): the two imagined heads' first-layer weight
        gradients are then one (2U, F) matrix that a single GEMM over their joint dy writes (ops.PairFirstFn)."""
        names = list(self._named_params)
        prms = list(self._named_params.values())
        idx = {id(p): i for i, p in enumerate(prms)}
        order = list(range(len(names)))
        self._pair_first = False
        if not (PAIR_FIRST and self.actor.mlp.n >= 1 and self.value.mlp.n >= 1):
            return order
        ia = idx.get(id(self.actor.mlp._mods[0][0].weight))
        iv = idx.get(id(self.value.mlp._mods[0][0].weight))
        act = [i for i, n in enumerate(names) if n.startswith("actor.")]
        if ia is not None and iv is not None and act and iv == act[-1] + 1 and \
                act == list(range(act[0], act[-1] + 1)) and prms[ia].shape == prms[iv].shape:
            order = [i for i in order if i != ia]
            order.insert(order.index(act[-1]) + 1, ia)
            self._pair_first = True
        return order

    def _grad_buckets(self):
        """Data parallel: the gradient arena split into all-reduce buckets by the phase after which each parameter's
        gradient is final (_update_graphed), as merged contiguous arena ranges:
          heads — world-model heads, projector / decoder / prototypes: M1 (main);
          ac    — actor and value heads: S2 (side; the replay-value part of the value head is deferred into S2);
          rssm  — the RSSM: S3 (side: the scan's deferred weight gradients; the prior's come from M1 before it);
          rest  — the encoder and anything unlisted: after M2c (main) and S4 (side)."""
        a = self._optimizer.arena
        pos = {id(p): i for i, p in enumerate(a.params)}
        group = {"actor": "ac", "value": "ac", "rssm": "rssm", "encoder": "rest"}
        out = {"heads": [], "ac": [], "rssm": [], "rest": []}
        for name, prm in self._named_params.items():
            i = pos[id(prm)]
            b = group.get(name.split(".")[0], "heads")
            out[b].append((a.offsets[i], a.offsets[i] + a.padded[i]))
        for b, rs in out.items():  # merged contiguous ranges (the arena's physical order need not be the named one)
            merged = []
            for lo, hi in sorted(rs):
                if merged and merged[-1][1] == lo:
                    merged[-1] = (merged[-1][0], hi)
                else:
                    merged.append((lo, hi))
            out[b] = merged
        return out

    def _allreduce_bucket(self, name, *events):
        """Sum all-reduce of one gradient bucket on the communication stream once `events` have fired (overlaps the
        phases still running on main / side; RCCL runs collectives in issue order, the same on every rank)."""
        with torch.cuda.stream(self._comm):
            for e in events:
                self._comm.wait_event(e)
            for lo, hi in self._buckets[name]:
                dist.all_reduce(self._optimizer.arena.grad[lo:hi])

    def _mark(self, tag):
        if self.marks is not None:
            self.marks(tag)

    def _main_tail(self, st):
        """phase M2d (main, after the first encoder stage's backward): deferred weight gradients moved off the side
        stream's tail (SDREAMER_DEFER_WM / SDREAMER_S4_MAIN)."""
        ops.flush_wgrads(st.get("wm_wgrads", []))
        ops.flush_wgrads(st.get("enc_wgrads_main", []))
        self._mark("main_tail")

    def _flush(self, wgrads, tag):
        """side phases S3 / S4: the deferred weight-gradient contractions, then a timeline mark."""
        ops.flush_wgrads(wgrads)
        self._mark(tag)

    def _core_forward(self, data, initial, seed, ro):
        """Graph phase P (main): preprocess, Polyak, zero_grad, encoder + posterior scan."""
        if self.marks is not None:
            self.marks.reset()
        p_data = self.preprocess(dict(data), enc_input=True)
        self._polyak()
        if self.rep_loss == "dreamerpro":  # replays run with ema_update_every == 1 and past update 0
            self._ema_apply(self._pro["frac"])
        if not self._step_zeroes:  # else the previous replay's optimizer step left the gradients zeroed
            self._optimizer.zero_grad()
        return self._ph_forward(p_data, initial, seed, ro)

    def _side_ac_metrics(self, st):
        """Graph phase S2 (side): the actor-critic phase, then the merged loss / metric vector. The metrics are built
        here, where the side stream has slack, instead of in front of the optimizer step (M3)."""
        self._ph_side_ac(st)
        post, mets = self._ph_finish(st)
        keys = [k for k, v in mets.items() if isinstance(v, (torch.Tensor, K.Stat))]
        mvec = K.metric_vector([mets[k] for k in keys])  # every metric of the update in one launch
        return post, keys, mvec

    def _core_step(self, st):
        """Graph phase M3 (main): the optimizer step."""
        # the arena was sum-all-reduced between the phase graphs (_update_graphed): the fused step reads the gradients
        # times 1 / world; DreamerPro's prototype gradient is also gated there (LaProp.gate)
        self._optimizer.grad_scale = 1.0 / self.world
        self._optimizer.launch_step()
        self._mark("optimizer")

    def _update_graphed(self, data, initial, seed, ro):
        """Replay of the update as eleven single-stream phases (captured once) joined by stream events:

            main: P (encoder, scan fwd) ─┬─ M1 (world-model heads, replay-value fwd) ─ wait(S1) ─ R (replay-value
                                         │   loss + bwd) ─┬─ M2a (scan bwd) ─┬─ M2b (encoder stages 2.. bwd) ─┬─ M2c
                                         │                │                  │                                │  (first
                                         │                │                  │   stage) ─ wait(side) ─ [grad all-reduce] ─ M3
            side:                        └─ S1 (imagination, heads, λ-returns) ─ wait(R) ─ S2 (value-head weight
                                                grads, ReturnEMA, actor / critic) ─ wait(M2a) ─ S3 (scan weight grads)
                                                ─ wait(M2b) ─ S4 (encoder stages 2.. weight grads)

        One graph per stream phase keeps every graph linear: the HIP runtime launches a linear graph as a batch
        (~0.5 ms of host time for the whole update) and the cross-stream edges become device-side event waits.
        A single two-stream graph instead costs ~12 ms of host time per launch, stalling on each cross-stream
        edge. Every graph has its own memory pool; tensors that cross phases are held by `self._gst`.

        Data parallel: a phase that exchanges data (Barlow statistics in M1, the returns gather for the global
        ReturnEMA in S2) is a chain graph → collective → graph (parallel.PhaseGraph); the collectives are issued
        eagerly on the phase's stream, in the same host order on every rank (M1's, then S2's after the R phase's
        launch), so RCCL's single stream never queues the world-model branch behind the actor-critic branch. The
        gradient arena is sum-all-reduced in four buckets (_grad_buckets) on a communication stream as soon as each
        bucket's last writer phase is done — WM heads after M1, actor / value after S2, RSSM after S3, encoder at the
        end — so only the encoder bucket's all-reduce sits between the joins and M3 (which scales the arena by
        1/world before AGC + LaProp)."""
        if self._graph is None:
            self._g_in = {k: v.clone() for k, v in data.items()}
            self._g_ro = ro
            self._g_init = tuple(t.clone() for t in initial)
            self._seed_dev = torch.zeros(1, dtype=torch.int64, device=self.device)
            main_cap = torch.cuda.Stream(device=self.device)
            side_cap = torch.cuda.Stream(device=self.device)
            # thread-local capture: RCCL's watchdog thread queries events while a multi-GPU phase is captured
            mode = "global" if self.world == 1 else "thread_local"
            torch.cuda.synchronize()

            def cap(fn, stream, fill=False):
                if not (fill and FILL_LDS):
                    return parallel.capture_phase(fn, stream, mode)
                old = nat.fns["sd_set_lds_pad"](FILL_LDS * 1024)  # returns the previous pad
                try:
                    return parallel.capture_phase(fn, stream, mode)
                finally:
                    nat.fns["sd_set_lds_pad"](max(old, 0))

            # zero_grad folded into the optimizer step (M3 zeroes what it reads); the gradients are zeroed eagerly
            # before a replay whenever something else wrote them (_grads_clean)
            self._step_zeroes = True
            gP, st = cap(lambda: self._core_forward(self._g_in, self._g_init, self._seed_dev, ro), main_cap)
            gS0, _ = cap(lambda: self._ph_side_prep(st), side_cap) if SIDE_PREP else (None, None)
            gS1, _ = cap(lambda: self._ph_side_returns(st), side_cap)
            gM1, _ = cap(lambda: self._ph_wm(st, defer=DEFER_WM), main_cap, fill=True)
            gR, _ = cap(lambda: self._ph_repval(st), main_cap)
            gM2a, _ = cap(lambda: self._ph_scan_bwd(st, defer=True), main_cap)
            if AC_DEFER:  # S2 captured before S3: its queued weight gradients are flushed at the start of S3
                st["rr"]["ac_wgrads"] = []
                gS2, (post, keys, mvec) = cap(lambda: self._side_ac_metrics(st), side_cap, fill=True)
            gS3, _ = cap(lambda: self._flush(st["rr"].get("ac_wgrads", []) + st["scan_wgrads"], "side:scan_wgrads"),
                         side_cap, fill=True)
            gM2b, _ = cap(lambda: self._ph_encoder_bwd_hi(st, defer=True), main_cap)
            if S4_MAIN:
                st["enc_wgrads_main"] = st["enc_wgrads"][:S4_MAIN]
                del st["enc_wgrads"][:S4_MAIN]
            gS4, _ = cap(lambda: self._flush(st["enc_wgrads"], "side:enc_wgrads"), side_cap, fill=True)
            gM2c, _ = cap(lambda: self._ph_encoder_bwd_lo(st), main_cap)
            gM2d = cap(lambda: self._main_tail(st), main_cap)[0] if (DEFER_WM or S4_MAIN) else None
            if not AC_DEFER:
                gS2, (post, keys, mvec) = cap(lambda: self._side_ac_metrics(st), side_cap, fill=True)
            self._optimizer.zero_grads_after = True
            gM3, _ = cap(lambda: self._core_step(st), main_cap)
            self._optimizer.zero_grads_after = False  # eager steps (step()) keep the PyTorch semantics
            self._grads_clean = False
            torch.cuda.synchronize()
            for g in (gS0, gP, gR, gM2a, gS3, gM2b, gS4, gM2c, gM2d, gM3):
                if g is gP and SIDE_PREP and SIDE_PREP_AT == "scan":
                    if g.n_collectives != 1:
                        raise RuntimeError("P should hold exactly the S0 fork point")
                elif g is not None and g.n_collectives:
                    raise RuntimeError("unexpected exchange step in a single-graph phase")
            self._graph = (gS0, gP, gS1, gM1, gR, gM2a, gS3, gM2b, gS4, gM2c, gM2d, gS2, gM3)
            self._gst, self._g_post, self._g_keys, self._g_mvec = st, post, keys, mvec
        if data is not None:
            for k, v in data.items():
                self._g_in[k].copy_(v)
            for dst, src in zip(self._g_init, initial):
                dst.copy_(src)
        # the update's noise seed into the graphs' device scalar as a pinned host-to-device copy (no fill kernel; the
        # caching host allocator keeps the pinned block until the copy has run)
        self._seed_dev.copy_(torch.tensor([int(seed) & 0x7FFFFFFFFFFFFFFF], dtype=torch.int64).pin_memory(),
                             non_blocking=True)
        if self.rep_loss == "dreamerpro":
            self._ema_updates += 1
            self._proto_gate.copy_(torch.tensor([0.0 if self._protos_frozen() else 1.0]).pin_memory()
                                   .reshape(self._proto_gate.shape), non_blocking=True)
        gS0, gP, gS1, gM1, gR, gM2a, gS3, gM2b, gS4, gM2c, gM2d, gS2, gM3 = self._graph
        caller = torch.cuda.current_stream()
        if STREAM_PRIO and self.use_side_stream:
            # the critical chain (P, S1, R, M2a..M2d, M3) on high-priority streams, the phases that fill its idle CUs
            # (M1 beside the imagination, S2-S4 beside the backward) on normal-priority ones: the dispatcher then
            # serves a waiting critical-chain workgroup before a filler one
            if self._prio_streams is None:
                mk = lambda pr: torch.cuda.Stream(device=self.device, priority=pr)  # noqa: E731
                self._prio_streams = (mk(-1), mk(-1), mk(0), mk(0))
            main, side, fill, side_fill = self._prio_streams
            main.wait_stream(caller)
        elif FILL_CUS and self.use_side_stream:
            if self._prio_streams is None:
                self._prio_streams = _cumask_streams(self.device)
            main, side = caller, self._side
            fill, side_fill = self._prio_streams
        else:
            main = caller
            side = self._side if self.use_side_stream else main
            fill, side_fill = main, side
        if gS0 is not None and SIDE_PREP_AT != "scan":  # S0 (weights and seed only) beside P: after the seed copy and
            # the last optimizer step (SIDE_PREP_AT=scan: forked from P itself, _fork_side_prep)
            if side is not main:
                side.wait_stream(main)
            with torch.cuda.stream(side):
                gS0.replay()
        with torch.cuda.stream(main):
            if not self._grads_clean:
                self._optimizer.zero_grad()
            gP.replay()
        if side is not main:
            side.wait_stream(main)
        if fill is not main:
            fill.wait_stream(main)
        k1 = gS1.first_collective()
        with torch.cuda.stream(side):
            gS1.replay(0, k1)
        with torch.cuda.stream(fill):
            gM1.replay()
            ev_m1 = torch.cuda.Event()
            ev_m1.record()
        dp = self.world > 1
        if dp and self._comm is None:
            self._comm = torch.cuda.Stream(device=self.device)
        with torch.cuda.stream(side):
            gS1.replay(k1)
            ev_s1 = torch.cuda.Event()
            ev_s1.record()
        if dp and not DEFER_WM:  # heads bucket final after M1 (else after M2d); issued after S1's returns gather so
            # RCCL's one communicator stream does not queue that gather (R waits on it) behind this all-reduce
            self._allreduce_bucket("heads", ev_m1)
        main.wait_event(ev_m1)
        main.wait_event(ev_s1)
        with torch.cuda.stream(main):
            gR.replay()
            ev_rep = torch.cuda.Event()
            ev_rep.record()
            gM2a.replay()
            ev_scan = torch.cuda.Event()
            ev_scan.record()
            if S2_AFTER_SCAN:
                ev_rep = ev_scan
            gM2b.replay()
            ev_enc = torch.cuda.Event()
            ev_enc.record()
            gM2c.replay()
            if gM2d is not None:
                gM2d.replay()
        ev_side = [None, None]
        if side_fill is not side:
            side_fill.wait_stream(side)
        with torch.cuda.stream(side_fill):
            side_fill.wait_event(ev_rep)
            gS2.replay()
            if dp:
                ev_side[0] = torch.cuda.Event()
                ev_side[0].record()
            side_fill.wait_event(ev_scan)  # S3: the scan's weight gradients, beside the encoder backward
            gS3.replay()
            if dp:
                ev_side[1] = torch.cuda.Event()
                ev_side[1].record()
            side_fill.wait_event(ev_enc)  # S4: encoder stages 2..'s weight gradients, beside the first stage's backward
            gS4.replay()
        if dp:  # bucketed sum all-reduce of the gradient arena, overlapping the backward phases still running
            ev_main, ev_s4 = torch.cuda.Event(), torch.cuda.Event()
            ev_main.record(main)
            self._allreduce_bucket("ac", ev_side[1] if AC_DEFER else ev_side[0])
            if DEFER_WM:  # the prior's img_net weight gradients are in M2d: the RSSM bucket also waits for main
                self._allreduce_bucket("rssm", ev_side[1], ev_main)
            else:
                self._allreduce_bucket("rssm", ev_side[1])
            ev_s4.record(side_fill)
            if DEFER_WM:
                self._allreduce_bucket("heads", ev_main)
            self._allreduce_bucket("rest", ev_main, ev_s4)
        if side_fill is not main:
            main.wait_stream(side_fill)
        if dp:
            main.wait_stream(self._comm)
        with torch.cuda.stream(main):
            gM3.replay()
        self._grads_clean = True
        if main is not caller:
            caller.wait_stream(main)
        self._slow_value_updates += 1
        self._optimizer.host_steps += 1
        self._updates += 1
        vec = self._g_mvec.clone()
        mets = {k: vec[i] for i, k in enumerate(self._g_keys)}
        mets["opt/lr"] = self._scheduler.get_lr()[0]
        mets["opt/grad_scale"] = 1.0
        return self._g_post, mets

    def _cal_grad(self, data, initial, seed=0, row_offset=0):
        """dreamer.py:453-671 (fp32). data: dict of (B, T, *) device tensors, image float in [0, 1].

        Same losses and gradients as the reference's single backward, scheduled as stream phases after the posterior
        scan (single GPU; data parallel stays on one stream):
          side — imagination, imagined heads, lambda-returns + ReturnEMA; later (after the replay-value backward) the
                 policy / value losses and their backward, overlapping the posterior backward;
          main — world-model head losses (prior/KL, representation, reward, continue) on detached LEAF copies of the
                 posterior and their backward down to the leaves, the replay-value forward; once the returns exist,
                 the replay-value loss (kept attached to the world model as in dreamer.py:652) and its backward; then
                 one backward from the posterior into the scan and the encoder.
        Gradient writes of the two streams touch disjoint parameters except the value head, whose two contributions
        are ordered by an event (replay value on main first, then the imagined value loss on side). Graph mode
        captures each phase separately (_update_graphed). Data parallel runs the same two streams; the exchange steps
        (parallel.collective) are issued on the stream of the phase that needs them."""
        self._grads_clean = False  # an eager backward writes the gradient arena
        st = self._ph_forward(data, initial, seed, row_offset)
        main = torch.cuda.current_stream()
        side = self._side if self.use_side_stream else main
        if side is not main:
            side.wait_stream(main)
            for t in (st["post_stoch"], st["post_deter"], st["feat_r"], data["reward"], data["is_last"],
                      data["is_terminal"]):
                t.record_stream(side)
        with torch.cuda.stream(side):
            self._ph_side_returns(st)
            ev_s1 = torch.cuda.Event()
            ev_s1.record()
        self._ph_wm(st)
        if side is not main:
            main.wait_event(ev_s1)
            for t in (st["ifeat"], st["iact"]):
                t.record_stream(main)
            for v in st["rr"].values():
                if isinstance(v, torch.Tensor):
                    v.record_stream(main)
        self._ph_repval(st)
        ev_rep = torch.cuda.Event()
        ev_rep.record()
        self._ph_posterior_bwd(st)
        with torch.cuda.stream(side):
            side.wait_event(ev_rep)
            self._ph_side_ac(st)
        if side is not main:
            main.wait_stream(side)
            for k in ("ac_losses", "ac_metrics"):
                for v in st[k].values():
                    v.record_stream(main)
        return self._ph_finish(st)

    def _ph_forward(self, data, initial, seed, ro):
        """main: encoder + posterior scan (dreamer.py:453-470); detached leaves for the two branches."""
        mk = self._mark
        mk("start")
        split = []  # the first encoder stage is backpropagated separately (_ph_encoder_bwd_lo)
        embed = self.encoder(data, split=split)
        mk("encoder_fwd")
        if SIDE_PREP and SIDE_PREP_AT == "scan" and parallel._active is not None:  # (graph capture of P only)
            parallel.collective(self._fork_side_prep)
        # the scan sees a leaf copy of embed: its backward stops there, so scan and encoder backward are separate
        # phases (_ph_scan_bwd / _ph_encoder_bwd)
        embed_l = embed.detach().requires_grad_(embed.requires_grad)
        post_stoch, post_deter, post_logit = self.rssm.observe(embed_l, data["action"], initial, data["is_first"],
                                                               seed=seed, row_offset=ro)
        mk("scan_fwd")
        leaves = [t.detach().requires_grad_(True) for t in (post_stoch, post_deter, post_logit)]
        ifeats = None
        if self._fused_imag_ok():
            # the posterior feat is written straight into the imagination's start slot (feats[0] of its time-major
            # (H1, N, F) buffer): the side stream's imagination starts from it without a copy
            B, T = post_deter.shape[:2]
            r = self.rssm
            ifeats = torch.empty(self.imag_horizon + 1, B * T, r.feat_size, dtype=torch.float32,
                                 device=post_deter.device)
            feat_l = ops.CatIntoFn.apply(leaves[0].reshape(B, T, r.flat_stoch), leaves[1],
                                         [ifeats[0].view(B, T, r.feat_size)])
        else:
            feat_l = self.rssm.get_feat(leaves[0], leaves[1])
        feat_r = feat_l.detach().requires_grad_(True)  # replay-value leaf (side stream)
        # every head reading the feat (reward, continue, projector, replay value) adds its input gradient into one
        # (B, T, F) buffer (ops.DxSink): the scan backward reads its two halves in place
        fsink = ops.DxSink(feat_l)
        ops.sink(feat_l, fsink)
        ops.sink(feat_r, fsink)
        return dict(data=data, initial=initial, seed=seed, ro=ro, embed=embed, embed_l=embed_l,
                    enc_split=split[0] if split else None, post_stoch=post_stoch,
                    post_deter=post_deter, post_logit=post_logit, leaves=leaves, feat_l=feat_l, feat_r=feat_r,
                    ifeats=ifeats, fsink=fsink)

    def _fork_side_prep(self):
        """P's split point after the encoder forward (SIDE_PREP_AT=scan), run on the host between P's two graphs at
        every replay: S0 on the side stream, after what main has queued so far (weights of the last step, the seed)."""
        g = self._graph
        if g is None or g[0] is None or not self.use_side_stream:
            return
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream())
        self._side.wait_event(ev)
        with torch.cuda.stream(self._side):
            g[0].replay()

    def _ph_side_prep(self, st):
        """side, beside the encoder forward (S0): what depends on the weights and the seed only — the imagination's
        noise and weight images (_imagine_prepare), the scan backward's transposed weights and the encoder's flipped
        conv weights (read by the backward phases)."""
        data = st["data"]
        B, T = data["action"].shape[:2]
        if self._fused_imag_ok():
            st["imag_prep"] = self._imagine_prepare(B * T, self.imag_horizon + 1, st["seed"], st["ro"] * T,
                                                    data["action"].device)
        if SIDE_PREP >= 2:
            st["scan_tr"] = self.rssm._bwd_tr = self.rssm.scan_bwd_weights()
            st["enc_flip"] = K.set_flip_cache(self.encoder.dgrad_weights())

    def _ph_side_returns(self, st):
        """side: imagination (dreamer.py:578-597), imagined heads, lambda-returns + ReturnEMA (598-636)."""
        data = st["data"]
        B, T = data["action"].shape[:2]
        N, H1 = B * T, self.imag_horizon + 1
        self._mark("side:fork")
        start = (st["post_stoch"].detach().reshape(N, self.rssm._stoch, self.rssm._discrete),
                 st["post_deter"].detach().reshape(N, self.rssm._deter))
        # actor layer 0's fp32 output of every imagined step, kept for the policy loss's actor forward (REUSE_H0)
        ah0 = torch.empty(H1, N, self.actor.mlp.out_dim, device=start[1].device) \
            if REUSE_H0 and self._fused_imag_ok() and not self.actor.mlp._symlog_inputs else None
        ifeat, iact = self._imagine_tm(start, H1, st["seed"], st["ro"] * T, actor_h0=ah0, feats=st.get("ifeats"),
                                       prep=st.get("imag_prep"))
        self._mark("side:imagine")
        rr = self._heads_returns(ifeat)
        rr["act_h0"] = ah0
        self._mark("side:heads_returns")
        st.update(ifeat=ifeat, iact=iact, rr=rr)

    def _ph_wm(self, st, defer=False):
        """main: world-model head losses and their backward down to the posterior leaves; the replay-value parts
        that do not need the imagined returns. defer: the heads' weight-gradient contractions are queued in
        st["wm_wgrads"] (graphed update: phase M2d)."""
        st["wm_wgrads"] = []
        # the scan backward's transposed weights and the encoder's flipped conv weights, while main has slack (it
        # waits for the imagined returns next): off the chain from the head losses to the encoder gradient
        if "scan_tr" not in st:  # (made by _ph_side_prep when that phase ran)
            st["scan_tr"] = self.rssm._bwd_tr = self.rssm.scan_bwd_weights()
            st["enc_flip"] = K.set_flip_cache(self.encoder.dgrad_weights())
        st["flags"] = self._episode_flags(st["data"])
        with ops.defer_wgrads(st["wm_wgrads"] if defer else None):
            st["wm_total"], st["wm_losses"], st["wm_metrics"] = self._wm_heads(st["data"], st["embed"], st["leaves"],
                                                                               st["feat_l"], st["seed"], st["ro"],
                                                                               st["initial"], st["flags"])
        self._mark("wm_heads")
        st["rv"] = self._repval_pre(st["data"], st["feat_r"], st["flags"])
        self._mark("repval_fwd")

    def _ph_repval(self, st):
        """main (after the returns): replay-value loss (dreamer.py:638-652, attached to the world model through
        feat_r) and its backward."""
        loss, rv_metrics, rret = self._repval_post(st["data"], st["rv"], st["rr"]["ret"])
        # the posterior backward needs only the feat gradient: the value head's weight / bias gradients are queued
        # and run at the start of the side stream's actor-critic phase (which accumulates into the same head next)
        st["rv_wgrads"] = []
        with ops.defer_wgrads(st["rv_wgrads"]):
            torch.autograd.backward(loss, self._repval_scale)
        self._mark("repval_bwd")
        st.update(repval=loss, rv_metrics=rv_metrics, rret=rret)

    def _ph_posterior_bwd(self, st):
        self._ph_scan_bwd(st)
        self._ph_encoder_bwd(st)

    def _ph_scan_bwd(self, st, defer=False):
        """main: posterior gradient = head-loss leaf grads + replay-value feat grad -> scan backward (to embed).
        defer: the scan's weight-gradient GEMMs are queued in st["scan_wgrads"] (graphed update: they run on the
        side stream beside the encoder backward, phase S3)."""
        SK = self.rssm.flat_stoch
        leaves = st["leaves"]
        self._mark("repval_wait")
        fs = st.get("fsink")
        g_feat = fs.buf if fs is not None and fs.written else None
        if st["feat_r"].grad is not None:  # a head outside the sink (none on the benched path)
            g_feat = st["feat_r"].grad if g_feat is None else g_feat + st["feat_r"].grad
        # the posterior gradient is leaf gradient + feat gradient: the feat gradient's halves go to the scan backward
        # as second summands (RSSM._bwd_extra), added where the scan reads them (no add launches); missing leaf
        # gradients stay None (the scan treats them as zero)
        g_stoch, g_deter, g_logit = (l.grad for l in leaves)
        if g_feat is not None:
            if self.rssm.takes_extra_grads(g_feat.shape[0]):
                self.rssm._bwd_extra = (g_feat[..., :SK], g_feat[..., SK:])
            else:
                g_stoch = g_feat[..., :SK].reshape(leaves[0].shape) + (0 if g_stoch is None else g_stoch)
                g_deter = g_feat[..., SK:] + (0 if g_deter is None else g_deter)
        outs = [(o, g) for o, g in zip((st["post_stoch"], st["post_deter"], st["post_logit"]), (g_stoch, g_deter, g_logit))
                if g is not None]
        st["scan_wgrads"] = []
        if not outs:  # nothing reads the posterior (no gradient): the extra summands alone drive the scan backward
            outs = [(st["post_logit"], torch.zeros_like(st["post_logit"]))]
        if defer:
            with ops.defer_wgrads(st["scan_wgrads"]):
                torch.autograd.backward([o for o, _ in outs], [g for _, g in outs])
        else:
            torch.autograd.backward([o for o, _ in outs], [g for _, g in outs])
        self.rssm._bwd_tr = None
        self._mark("scan_bwd")

    def _ph_encoder_bwd(self, st):
        """main: encoder backward from the scan's embed gradient."""
        self._ph_encoder_bwd_hi(st)
        self._ph_encoder_bwd_lo(st)

    def _ph_encoder_bwd_hi(self, st, defer=False):
        """main: encoder stages 2.. backward (the data-gradient chain) down to the first stage's output leaf.
        defer: their bwd-weight contractions are queued in st["enc_wgrads"] (graphed update: side phase S4, beside
        the first stage's backward)."""
        g = st["embed_l"].grad
        st["enc_wgrads"] = []
        if g is not None:
            if defer:
                with ops.defer_wgrads(st["enc_wgrads"]):
                    st["embed"].backward(g)
            else:
                st["embed"].backward(g)
        K.clear_flip_cache()

    def _ph_encoder_bwd_lo(self, st):
        """main: the first encoder stage's backward (weight gradients only)."""
        sp = st["enc_split"]
        if sp is not None and sp[1].grad is not None:
            sp[0].backward(sp[1].grad)
        self._mark("encoder_bwd")

    def _ph_side_ac(self, st):
        """side: the replay-value loss's deferred value-head weight gradients, ReturnEMA + advantage, policy / value
        losses on the imagined trajectories and their backward."""
        ops.flush_wgrads(st["rv_wgrads"])
        self._slow_values(st["ifeat"], st["rr"])
        self._returns_norm(st["rr"])
        st["ac_losses"], st["ac_metrics"] = self._ac_losses(st["ifeat"], st["iact"], st["rr"])
        with torch.no_grad():  # replay-value statistics (dreamer.py:649-651), off the main stream's critical path
            st["ac_metrics"].update(_tstats(st["rret"], "ret_replay"))
            st["ac_metrics"].update(_tstats(st["rv"]["value"], "value_replay"))
            st["ac_metrics"].update(_tstats(st["rv"]["slow_value"], "slow_value_replay"))
        self._mark("side:actor_critic")

    def _ph_finish(self, st):
        losses, metrics = dict(st["wm_losses"]), dict(st["wm_metrics"])
        self._mark("join")
        losses["repval"] = st["repval"]
        losses.update(st["ac_losses"])
        metrics.update(st["rv_metrics"])
        metrics.update(st["ac_metrics"])
        total = K.Stat(st["wm_total"].detach())
        for k, v in losses.items():
            if k in ("repval", "policy", "value"):
                total = total + K.Stat(v.detach(), scale=self._loss_scales[k])
        metrics.update({f"loss/{k}": v.detach() for k, v in losses.items()})
        metrics["opt/loss"] = total
        rr = st["rr"]
        self._last = dict(embed=st["embed"], post_logit=st["post_logit"], prior_logit=self._prior_logit,
                          imag_feat_tm=st["ifeat"], imag_action_tm=st["iact"], ret=rr["ret"], rret=st["rret"])
        return (st["post_stoch"], st["post_deter"]), metrics

    def _wm_heads(self, data, embed, leaves, feat, seed=0, ro=0, initial=None, flags=None):
        """World-model losses (dreamer.py:453-576) on the posterior leaves, backward down to the leaves. flags: the
        batch's (last, term, cont) f32 tensors (K.episode_flags), else derived here."""
        losses, metrics = {}, {}
        B, T = data["action"].shape[:2]
        post_stoch, post_deter, post_logit = leaves
        prior_logit = self.rssm.prior(post_deter)
        self._prior_logit = prior_logit
        dyn_loss, rep_loss = self.rssm.kl_loss(post_logit, prior_logit, self.kl_free)
        # the loss dict's per-row terms and scalars, reduced and weighted by one LossTermsFn launch below: name ->
        # (rows or scalar, coefficient of its mean)
        terms = {"dyn": (dyn_loss, 1.0), "rep": (rep_loss, 1.0)}
        if self.rep_loss == "dreamer":
            recon = self.decoder(post_stoch, post_deter)
            for key, mode in recon.items():
                if key in self.decoder.cnn_shapes:
                    dist = (mode - data[key]) ** 2  # MSEDist(agg="sum"), distributions.py:146-155
                    losses[key] = dist.sum(list(range(2, dist.dim()))).mean()
                else:
                    d = (mode - K.symlog(data[key].contiguous())) ** 2.0  # SymlogDist mse, distributions.py:174-190
                    d = torch.where(d < 1e-8, torch.zeros_like(d), d)
                    losses[key] = d.sum(list(range(2, d.dim()))).mean()
        elif self.rep_loss == "infonce":  # dreamer.py:533-542
            x1 = self.prj(feat).reshape(B * T, -1)
            losses["infonce"] = parallel.infonce(x1, embed.reshape(B * T, -1), self.world)
        elif self.rep_loss == "dreamerpro":  # dreamer.py:543-566
            losses.update(self._proto_losses(data, initial, seed, ro))
        else:
            x1 = self.prj(feat).reshape(B * T, -1)
            if self.r2_aug is not None:  # encoder on a randomly translated view, no gradient (dreamer.py:506-520)
                with torch.no_grad():
                    pad, same, bil = self.r2_aug
                    aug = {k: v for k, v in data.items() if k != "__enc_image"}  # the encoder re-forms its input
                    aug["image"] = K.random_translate(data["image"], pad, seed, ro, same, bil)
                    x2 = self.encoder(aug).reshape(B * T, -1)
            else:
                x2 = embed.reshape(B * T, -1).detach()
            losses["barlow"] = parallel.barlow(x1, x2, self.barlow_lambd, self.world)
        terms.update({k: (v, 1.0) for k, v in losses.items()})  # the representation loss(es), in dict order
        losses = {}
        rew_logits = self.reward(feat)
        terms["rew"] = (ops.TwoHotLogProbFn.apply(rew_logits, self.rbins, data["reward"].float()), -1.0)
        cont = flags[2] if flags is not None else 1.0 - data["is_terminal"].float()
        terms["con"] = (ops.BernoulliLogProbFn.apply(self.cont(feat), cont), -1.0)
        S = self.rssm._stoch
        metrics["dyn_entropy"] = K.Stat(self.rssm.entropy_terms(prior_logit), scale=S)
        metrics["rep_entropy"] = K.Stat(self.rssm.entropy_terms(post_logit), scale=S)
        names = list(terms)
        xs = [terms[k][0].reshape(-1) if terms[k][0].dim() == 0 else terms[k][0] for k in names]
        wm_total, vec = ops.LossTermsFn.apply([terms[k][1] for k in names], [self._loss_scales[k] for k in names],
                                              *xs)
        losses = {k: vec[i] for i, k in enumerate(names)}
        torch.autograd.backward(wm_total, self._unit(wm_total.device))  # the seed gradient without a fill launch
        return wm_total, losses, metrics

    def _proto_losses(self, data, initial, seed, ro):
        """DreamerPro (dreamer.py:543-566, 731-750): the batch doubled under two random translations (shifts
        indexed by the global augmented row: copy 1 rows ro.., copy 2 rows B_global + ro..), targets from the EMA
        encoder, and a second posterior scan (noise stream OBS_AUG, same global-row indexing) whose backward joins
        the world-model backward. Rows are independent in the scan, so the two copies run as two scans."""
        c = self._pro
        B, T = data["action"].shape[:2]
        Bg = B * self.world
        with torch.no_grad():
            aug = {k: torch.cat([v, v], 0) for k, v in data.items() if k != "__enc_image"}
            img = data["image"]
            aug["image"] = torch.cat([K.random_translate(img, c["pad"], seed, ro, c["same"], c["bilinear"]),
                                      K.random_translate(img, c["pad"], seed, Bg + ro, c["same"], c["bilinear"])], 0)
            ema = self._ema_obs_proj(self._ema_encoder(aug))
            ema = ema / ema.norm(dim=-1, keepdim=True).clamp_min(1e-12)
        embed = self.encoder(aug)
        outs = [self.rssm.observe(embed[h], data["action"], initial, data["is_first"], seed=seed, row_offset=off,
                                  stream_id=STREAM_OBS_AUG)
                for h, off in ((slice(0, B), ro), (slice(B, 2 * B), Bg + ro))]
        post_stoch = torch.cat([outs[0][0], outs[1][0]], 0)
        post_deter = torch.cat([outs[0][1], outs[1][1]], 0)
        return self._proto_loss(post_stoch, post_deter, embed, ema)

    def _sinkhorn(self, scores):  # dreamer.py:764-790: log-space Sinkhorn-Knopp over (K, N)
        c = self._pro
        Kp = scores.shape[0]
        lq = torch.log_softmax(scores.reshape(-1) / c["eps"], 0).view(Kp, -1)
        N = lq.shape[1]
        for _ in range(c["iters"]):
            lq = lq - torch.logsumexp(lq, 1, keepdim=True) - math.log(Kp)
            lq = lq - torch.logsumexp(lq, 0, keepdim=True) - math.log(N)
        return torch.exp(lq + math.log(N)).view(scores.shape)

    def _proto_loss(self, post_stoch, post_deter, embed, ema):
        """Dreamer.proto_loss (dreamer.py:792-843). The Sinkhorn targets balance each augmented half over the
        GLOBAL batch: under data parallelism each half's EMA projections are gathered (rank order = global row
        order), every rank runs the same Sinkhorn and keeps its own columns."""
        c = self._pro
        w, tau = c["warm_up"], c["tau"]
        B2, T = embed.shape[:2]
        B = B2 // 2
        protos = F.normalize(self._prototypes, p=2, dim=-1)

        def scores(x, pr):  # unit rows (n, T, Pd) -> (K, n, T - warm_up)
            n = x.shape[0]
            return ops.MatmulNTFn.apply(x.reshape(n * T, -1), pr).view(n, T, -1).permute(2, 0, 1)[:, :, w:]

        obs = self.obs_proj(embed)
        obs_norm = obs.norm(dim=-1)
        obs_logits = F.log_softmax(scores(F.normalize(obs, p=2, dim=-1), protos) / tau, dim=0)
        o1, o2 = obs_logits.chunk(2, dim=1)
        with torch.no_grad():
            pr = protos.detach()
            lo = self.rank * B if self.world > 1 else 0
            t = []
            for half in (ema[:B], ema[B:]):
                q = self._sinkhorn(scores(parallel.gather_returns(half.contiguous(), self.world), pr))
                t.append(q[:, lo:lo + B])
            t1, t2 = t
        targets = torch.cat([t1, t2], 1)
        feat = self.feat_proj(self.rssm.get_feat(post_stoch, post_deter))
        feat_norm = feat.norm(dim=-1)
        feat_logits = F.log_softmax(scores(F.normalize(feat, p=2, dim=-1), protos) / tau, dim=0)
        swav = -0.5 * (t2 * o1).sum(0).mean() - 0.5 * (t1 * o2).sum(0).mean()
        temp = -(targets * feat_logits).sum(0).mean()
        norm = ((obs_norm - 1) ** 2).mean() + ((feat_norm - 1) ** 2).mean()
        return {"swav": swav, "temp": temp, "norm": norm}

    def _unit(self, device):
        """device 1.0 (created once, outside any capture): the seed gradient of a loss total"""
        if self._one is None:
            self._one = torch.ones((), dtype=torch.float32, device=device)
        return self._one

    @staticmethod
    def _episode_flags(data):
        """(last, term, cont = 1 - term) as f32 (B, T): one launch from the replay's bool flags"""
        il, it = data["is_last"], data["is_terminal"]
        if il.dtype == torch.bool and it.dtype == torch.bool and il.is_contiguous() and it.is_contiguous():
            return K.episode_flags(il, it)
        B, T = data["action"].shape[:2]
        last, term = il.float().reshape(B, T), it.float().reshape(B, T)
        return last, term, 1.0 - term

    def _repval_pre(self, data, feat_r, flags=None):
        """Replay-value parts that do not need the imagined returns (dreamer.py:638-652): value / slow-value modes on
        the replay posterior, the value head forward (with grad) and the slow-target log-prob. The value head runs on
        every posterior step (the loss reads its first T - 1 in place: no copy of feat[:, :-1], no slice backward)."""
        B, T = data["action"].shape[:2]
        N = B * T
        vd = self.value(feat_r)
        with torch.no_grad():
            fd = feat_r.detach().reshape(N, -1)
            # _frozen_value aliases value (dreamer.py:642 vs 648): its mode is read off the logits the loss's forward
            # computes anyway (same f32 kernels, so the same values), not from a second forward of the head
            value = K.twohot_mode(vd.detach().reshape(N, -1), self.vbins).view(B, T)
            slow_value = K.twohot_mode(self._slow_value.logits_nograd(fd), self.vbins).view(B, T)
        last, term, _ = flags if flags is not None else self._episode_flags(data)
        reward = data["reward"].float().reshape(B, T)
        return dict(value=value, slow_value=slow_value, vd=vd, last=last, term=term,
                    reward=reward if reward.is_contiguous() else reward.contiguous())

    def _repval_post(self, data, rv, ret):
        """Replay lambda-return bootstrapped from the imagined return (dreamer.py:645) and the replay-value loss."""
        B, T = data["action"].shape[:2]
        H = self.imag_horizon
        disc = 1 - 1 / self.horizon
        with torch.no_grad():
            # boot = imag ret[:, 0]: ret is (N, H) with N = (b, t)
            rret = K.lambda_return(rv["reward"], ret, disc, self.lamb, term=rv["term"], last=rv["last"],
                                   boot_row_stride=T * H, boot_t_stride=H)  # (B, T-1)
        loss = ops.RepvalLossFn.apply(rv["vd"], self.vbins, rret, rv["slow_value"], rv["last"])
        return loss, {}, rret  # the replay statistics are logged from the side stream (_ph_side_ac)

    @torch.no_grad()
    def _heads_returns(self, ifeat):
        """Imagined reward / continue / value / slow-value heads (dreamer.py:598-622) and the lambda-returns. The
        ReturnEMA quantiles and the advantage (dreamer.py:623-636) are only read by the policy / value losses, so they
        run at the start of the side stream's actor-critic phase (_returns_norm), off the replay-value path."""
        H1, N = ifeat.shape[:2]
        dev = ifeat.device
        flat = ifeat.reshape(H1 * N, -1)
        # frozen heads on the imagined trajectories: split-bf16 contractions (no sampled index depends on them), the
        # four first layers as one batched launch
        firsts = []
        # the slow critic feeds only the value loss's target and a metric (dreamer.py:606,616,666): with SLOW_IN_S2 it
        # runs in the actor-critic phase (_slow_values), off the path from the imagination to the lambda-returns
        heads = (self.reward, self.cont, self.value) + (() if SLOW_IN_S2 else (self._slow_value,))
        outs = heads_nograd(heads, flat, True, firsts_out=firsts)
        l_rew, l_cont, l_val = outs[:3]
        i_rew = K.twohot_mode(l_rew, self.rbins).view(H1, N)
        i_contl = l_cont.reshape(H1, N)  # a column of the fused output layer's padded logits
        i_val = K.twohot_mode(l_val, self.vbins).view(H1, N)
        i_slow = None if SLOW_IN_S2 else K.twohot_mode(outs[3], self.vbins).view(H1, N)
        disc = 1 - 1 / self.horizon
        i_cont = torch.empty(N, H1, device=dev)
        weight = torch.empty(N, H1, device=dev)
        # the time-major head outputs read in place through (N, H1) transposed views
        ret = K.lambda_return(i_rew.t(), i_val, disc, self.lamb, cont_logit=i_contl.t(), cont_out=i_cont,
                              weight_out=weight, boot_row_stride=1, boot_t_stride=N)  # (N, H)
        # the value head's first layer on the imagined feats, the same contraction the value loss's forward needs
        # (_frozen_value aliases value; the weights change only at the optimizer step)
        val_h0 = firsts[0][2] if (firsts and REUSE_H0) else None
        return dict(ret=ret, weight=weight, i_cont=i_cont, i_rew=i_rew, i_val=i_val, i_slow=i_slow, val_h0=val_h0)

    @torch.no_grad()
    def _slow_values(self, ifeat, rr):
        """The slow critic's mode on the imagined trajectories (dreamer.py:593 _frozen_slow_value(imag_feat).mode()),
        when _heads_returns left it out (SLOW_IN_S2)."""
        if rr.get("i_slow") is None:
            H1, N = ifeat.shape[:2]
            (l_slow,) = heads_nograd((self._slow_value,), ifeat.reshape(H1 * N, -1), True)
            rr["i_slow"] = K.twohot_mode(l_slow, self.vbins).view(H1, N)

    @torch.no_grad()
    def _returns_norm(self, rr):
        """ReturnEMA over every rank's returns (global quantiles, dreamer.py:623-627) and the advantage (628-636)."""
        ret_all = parallel.gather_returns(rr["ret"], self.world)
        ret_offset, ret_scale = self.return_ema(ret_all)
        rr.update(ret_offset=ret_offset, ret_scale=ret_scale)  # the advantage is formed inside the AC loss launch

    def _ac_losses(self, ifeat, iact, rr):
        """Policy and value losses on the imagined trajectories (dreamer.py:653-671) and their backward."""
        losses, metrics = {}, {}
        H1, N = ifeat.shape[:2]
        H = H1 - 1
        ret, weight, i_slow = rr["ret"], rr["weight"], rr["i_slow"]
        xh = ifeat[:H].reshape(H * N, -1)
        a_h0, v_h0 = rr.get("act_h0"), rr.get("val_h0")
        pair = None
        if self._pair_first and a_h0 is not None and v_h0 is not None:
            # both first layers given (the actor's from the imagination, the value head's from the imagined heads):
            # their weight gradients are one GEMM over the joint dy (ops.PairFirstFn)
            pair = pair_forward_from_first(self.actor, self.value, xh, a_h0[:H].reshape(H * N, -1), v_h0[:H * N],
                                           fast=True)
        if pair is not None:
            pl, vl = pair
        elif a_h0 is not None:  # layer 0 from the imagination (fp32), layers 1.. and the output on split-bf16
            pl = self.actor.forward_from_first(xh, a_h0[:H].reshape(H * N, -1), fast=True)
        else:
            pl = self.actor(xh, fast=True)
        if self.act_discrete:
            logpi, ent = ops.OneHotLogProbEntFn.apply(pl, iact[:H].reshape(H * N, -1),
                                                       float(self.config.actor.dist.unimix_ratio))
        else:
            d = self.config.actor.dist
            logpi, ent = ops.BNormalLogProbEntFn.apply(pl, iact[:H].reshape(H * N, -1), float(d.min_std),
                                                        float(d.max_std))
        if pair is None:
            if v_h0 is not None:  # layer 0 from the imagined heads' batched launch (its first H * N rows)
                vl = self.value.forward_from_first(xh, v_h0[:H * N], fast=True)
            else:
                vl = self.value(xh, fast=True)
        # policy (dreamer.py:653-660) and value (661-671) losses and the advantage (628-636): one launch each way
        total, losses["policy"], losses["value"], adv = ops.ImagACLossFn.apply(
            vl, logpi, ent, self.vbins, ret, i_slow[:H], weight, rr["i_val"], rr["ret_scale"], self.act_entropy,
            self._loss_scales["policy"], self._loss_scales["value"])
        rr["adv"] = adv
        with ops.defer_wgrads(rr["ac_wgrads"]) if "ac_wgrads" in rr else contextlib.nullcontext():
            torch.autograd.backward(total, self._unit(total.device))
        with torch.no_grad():
            # mean((ret - offset) / scale) as (mean(ret) - offset) / scale, resolved with the other metrics
            metrics["ret"] = K.Stat(ret, sub=rr["ret_offset"].reshape(1), div=rr["ret_scale"].reshape(1))
            metrics["ret_005"] = K.Stat(self.return_ema.ema_vals[0:1])
            metrics["ret_095"] = K.Stat(self.return_ema.ema_vals[1:2])
            metrics["adv"] = K.Stat(adv)
            metrics["adv_std"] = K.Stat(adv, K.STAT_STD)
            metrics["con"] = K.Stat(rr["i_cont"])
            metrics["rew"] = K.Stat(rr["i_rew"])
            metrics["val"] = K.Stat(rr["i_val"])
            metrics["tar"] = K.Stat(ret)
            metrics["slowval"] = K.Stat(i_slow)
            metrics["weight"] = K.Stat(weight)
            metrics["action_entropy"] = K.Stat(ent.detach())
            metrics.update(_tstats(iact, "action"))
        return losses, metrics

    @torch.no_grad()
    def _fused_imag_ok(self):
        r, a = self.rssm, self.actor
        if not FUSED_IMAG or a.mlp._symlog_inputs or a.mlp.out_dim != r._hidden or r._hidden != 256:
            return False
        if a.dist_name not in ("bounded_normal", "onehot") or r._deter % r._blocks or r._deter > 4096:
            return False
        A = self.act_dim
        return (r._deter // r._blocks) % 32 == 0 and r.flat_stoch % 64 == 0 and r._discrete in (16, 32) and \
            (A <= 16 if self.act_discrete else 2 * A <= 32) and 1 <= a.mlp.n <= 4 and 1 <= r._img_layers <= 4 and \
            a.last.weight.shape[0] <= 32

    def _imagine_prepare(self, N, H1, seed, row_offset, device):
        """The imagination's descriptor, workspace and everything in it that depends on the weights and the seed only:
        the drawn-ahead noise (sd_imagine_noise) and the pre-split / transposed weight images (sd_imagine_prep). The
        graphed update runs it as its own side-stream phase beside the encoder forward (S0), off the chain from the
        posterior to the imagined returns; _imagine_fused(prep=...) then runs the steps."""
        r, a = self.rssm, self.actor
        P = r._p()
        d = nat.ImagineDesc()
        d.N, d.H1, d.D, d.U, d.SK, d.Kd, d.G, d.A = N, H1, r._deter, r._hidden, r.flat_stoch, r._discrete, r._blocks, \
            self.act_dim
        d.act_discrete, d.actor_layers, d.img_layers = int(self.act_discrete), a.mlp.n, r._img_layers
        dist = self.config.actor.dist
        d.eps, d.unimix = K.EPS, r._unimix_ratio
        if self.act_discrete:
            d.act_unimix = float(dist.unimix_ratio)
        else:
            d.min_std, d.max_std = float(dist.min_std), float(dist.max_std)
        d.seed, d.seed_ptr = K.seed_args(seed)
        d.stream_img, d.stream_act, d.row_offset = STREAM_IMG, STREAM_ACT, int(row_offset)
        for i, (lin, norm) in enumerate(a.mlp._mods):
            d.Wa[i], d.ba[i], d.na[i] = lin.weight.data_ptr(), lin.bias.data_ptr(), norm.weight.data_ptr()
        wo = a.last.weight.contiguous()  # (2A or A, U): the action tile zero-fills its rows past them
        d.Wao, d.bao = wo.data_ptr(), a.last.bias.data_ptr()
        for k in ("W0", "b0", "n0", "W1", "b1", "n1", "W2", "b2", "n2", "Wh", "bh", "nh", "Wg", "bg"):
            setattr(d, k, P[k].data_ptr())
        mods, last = r._img_mods()
        for i, (lin, norm) in enumerate(mods):
            d.Wi[i], d.bi[i], d.ni[i] = lin.weight.data_ptr(), lin.bias.data_ptr(), norm.weight.data_ptr()
        d.Wl, d.bl = last.weight.data_ptr(), last.bias.data_ptr()
        nwork = nat.fns["sd_imagine_work_floats"](ctypes.addressof(d))
        if nwork < 0:
            raise nat.NativeError(f"sd_imagine_work_floats failed with status {nwork}")
        work = torch.empty(nwork, dtype=torch.float32, device=device)
        d.work = work.data_ptr()
        noise = None
        if IMAG_NOISE and H1 > 1:  # the prior samples' and actions' noise drawn in one full-chip launch up front
            noise = torch.empty((H1 - 1) * N * r.flat_stoch + H1 * N * self.act_dim, dtype=torch.float32, device=device)
            nact = noise[(H1 - 1) * N * r.flat_stoch:]
            d.noise_img, d.noise_act = noise.data_ptr(), nact.data_ptr()
            nat.call("sd_imagine_noise", ctypes.addressof(d), noise.data_ptr(), nact.data_ptr(), K.stream())
        nat.call("sd_imagine_prep", ctypes.addressof(d), K.stream())
        d.prepped = 1
        return dict(desc=d, work=work, wo=wo, P=P, noise=noise, N=N, H1=H1)

    def _imagine_fused(self, feats, actions, H1, seed, row_offset, chunks=None, keep=None, actor_h0=None, prep=None):
        """sd_imagine_run (csrc/img.hip): feats[0] holds the start state. chunks: step boundaries [t0, t1, ..., H1];
        the steps run as one launch sequence per chunk with an event recorded after each (returned), so consumers on
        other streams can start on a chunk's feats while the next chunk is imagined. prep: _imagine_prepare's result
        for this shape and seed (made here when None)."""
        N = feats.shape[1]
        if prep is None:
            prep = self._imagine_prepare(N, H1, seed, row_offset, feats.device)
        assert prep["N"] == N and prep["H1"] == H1, (prep["N"], prep["H1"], N, H1)
        d = prep["desc"]
        d.feats, d.actions = feats.data_ptr(), actions.data_ptr()
        if IMAG_TRACE is not None:  # measurement aid (tools/imag_trace.py, a -DSD_SCAN_TRACE build of the library)
            d.trace = IMAG_TRACE.data_ptr()
        d.actor_h0 = None
        if actor_h0 is not None:
            assert actor_h0.is_contiguous() and tuple(actor_h0.shape) == (H1, N, self.rssm._hidden), actor_h0.shape
            d.actor_h0 = actor_h0.data_ptr()
        bounds = list(chunks) if chunks else [0, H1]
        if keep is not None:  # measurement aid (bench.py): the descriptor and every buffer it points to
            keep.update(desc=d, work=prep["work"], wo=prep["wo"], feats=feats, actions=actions, P=prep["P"],
                        noise=prep["noise"])
        events = []
        for t0, t1 in zip(bounds[:-1], bounds[1:]):
            d.t_begin, d.t_end = int(t0), int(t1)
            nat.call("sd_imagine_run", ctypes.addressof(d), K.stream())
            if chunks:
                ev = torch.cuda.Event()
                ev.record()
                events.append(ev)
        return events

    def _imagine_tm(self, start, H1, seed, row_offset=0, chunks=None, actor_h0=None, feats=None, prep=None):
        """Dreamer._imagine (dreamer.py:673-692), time-major: feats (H1, N, F), actions (H1, N, A).
        The reference's last img_step (whose output is discarded) is skipped. With `chunks` (step boundaries) returns
        (feats, actions, events) with one event per chunk (see _imagine_fused). feats (fused path): a buffer whose
        feats[0] already holds the start state [stoch | deter] (_ph_forward writes it there)."""
        stoch, deter = start
        N = deter.shape[0]
        SK = self.rssm.flat_stoch
        preset = feats is not None and self._fused_imag_ok()
        if not preset:
            feats = torch.empty(H1, N, self.rssm.feat_size, dtype=torch.float32, device=deter.device)
        actions = torch.empty(H1, N, self.act_dim, dtype=torch.float32, device=deter.device)
        s = stoch.reshape(N, SK)
        h = deter
        if self._fused_imag_ok():
            if not preset:
                feats[0, :, :SK] = s
                feats[0, :, SK:] = h
            events = self._imagine_fused(feats, actions, H1, seed, row_offset, chunks, actor_h0=actor_h0, prep=prep)
            return (feats, actions, events) if chunks else (feats, actions)
        s, h = s.contiguous(), h.contiguous()
        for t in range(H1):
            feats[t, :, :SK] = s
            feats[t, :, SK:] = h
            logits = self.actor.logits_nograd(feats[t])
            actions[t] = self._sample_action(logits, seed, t, row_offset, STREAM_ACT)
            if t == H1 - 1:
                break
            h = self.rssm._deter_fwd(s, h, K.action_norm(actions[t]))
            s, _ = self.rssm._prior_nograd(h, seed, t, row_offset, STREAM_IMG)
        if chunks:
            ev = torch.cuda.Event()
            ev.record()
            return feats, actions, [ev] * (len(chunks) - 1)
        return feats, actions

    @torch.no_grad()
    def _imagine(self, start, imag_horizon, seed=0, row_offset=0):
        """Reference-layout wrapper: (N, H1, F), (N, H1, A)."""
        f, a = self._imagine_tm(start, imag_horizon, seed, row_offset)
        return f.transpose(0, 1), a.transpose(0, 1)

    @torch.no_grad()
    def _lambda_return(self, last, term, reward, value, boot, disc, lamb):  # dreamer.py:694-707
        N, T = reward.shape[:2]
        r = K.lambda_return(reward.reshape(N, T).float().contiguous(), boot.reshape(N, T).float().contiguous(),
                            disc, lamb, term=term.reshape(N, T).float().contiguous(),
                            last=last.reshape(N, T).float().contiguous())
        return r.unsqueeze(-1)

    # ------------------------------------------------------------------ checkpoint layout (train.py:126-130)
    _FROZEN = (("encoder", "_frozen_encoder"), ("rssm", "_frozen_rssm"), ("reward", "_frozen_reward"),
               ("cont", "_frozen_cont"), ("actor", "_frozen_actor"), ("value", "_frozen_value"),
               ("_slow_value", "_frozen_slow_value"))

    def to_ref_layout(self, param, t):
        """A tensor shaped like trainable parameter `param` (e.g. its .grad), viewed in the reference's layout."""
        i = [id(p) for p in self._named_params.values()].index(id(param))
        lay = self._ref_layouts[i]
        return t if lay is None else lay[0](t)

    def state_dict(self, *args, **kwargs):
        sd = super().state_dict(*args, **kwargs)
        extra = OrderedDict()
        for src, dst in self._FROZEN:
            for k, v in sd.items():
                if k.startswith(src + "."):
                    extra[dst + k[len(src):]] = v
        sd.update(extra)
        return sd

    def load_state_dict(self, state_dict, strict=True):
        sd = OrderedDict((k, v) for k, v in state_dict.items() if not k.startswith("_frozen_"))
        out = super().load_state_dict(sd, strict=strict)
        self._optimizer.arena.rebind()
        a = self._optimizer.arena
        pos = {id(p): i for i, p in enumerate(a.params)}
        for p, sp in zip([p for n, p in self._named_params.items() if n.startswith("value.")],
                         self._slow_value.parameters()):
            j = pos[id(p)]
            o = a.offsets[j] - self._v_lo
            if sp.data.data_ptr() != self._slow_arena[o:o + a.sizes[j]].data_ptr():
                self._slow_arena[o:o + a.sizes[j]].copy_(sp.data.reshape(-1))
                sp.data = self._slow_arena[o:o + a.sizes[j]].view(sp.shape)
        return out
