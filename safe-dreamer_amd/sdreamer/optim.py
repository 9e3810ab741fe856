"""LaProp + AGC over a flat parameter arena (reference: utils/optim/laprop.py, utils/optim/agc.py).

All trainable parameters of the Dreamer are re-homed into ONE contiguous fp32 arena (param.data becomes a view),
and their gradients into a second arena (param.grad views). That gives:
  * one fused HIP step (sd_agc_laprop_step): per-tensor AGC norms, clip, LaProp moments and the parameter update;
  * one buffer to all-reduce under data parallelism (RCCL over xGMI) — no per-tensor collectives;
  * one memset to zero the gradients.
`LaProp` subclasses torch.optim.Optimizer only so checkpoint tooling that walks attributes for optimizers
(tools.recursively_collect_optim_state_dict, tools.py:298-318) finds it; its state_dict uses the reference's
per-parameter state keys {step, exp_avg, exp_avg_lr_1, exp_avg_lr_2, exp_avg_sq} (laprop.py:62-70).
"""
from __future__ import annotations

import torch

from . import _native as nat
from . import kernels as K

CHUNK = 16384  # elements per optimiser block (one 256-thread workgroup streams one chunk of one tensor)


class FlatArena:
    """order: optional physical placement (a permutation of the parameter indices); tensor i stays index i for the
    optimizer state, the chunk tables and the checkpoint, only its offset follows the order. Used to put two layers
    whose weight gradients one GEMM writes back to back (the imagined actor's and value head's first layers)."""

    def __init__(self, params, device, order=None):
        self.params = list(params)
        self.sizes = [p.numel() for p in self.params]
        order = list(range(len(self.params))) if order is None else list(order)
        if sorted(order) != list(range(len(self.params))):
            raise ValueError("FlatArena order must be a permutation of the parameter indices")
        self.offsets = [0] * len(self.params)
        self.padded = [(n + 63) // 64 * 64 for n in self.sizes]  # 256-B aligned starts: float4-friendly views
        off = 0
        for i in order:
            self.offsets[i] = off
            off += self.padded[i]
        self.total = off
        self.data = torch.zeros(self.total, dtype=torch.float32, device=device)
        self.grad = torch.zeros(self.total, dtype=torch.float32, device=device)
        for p, o, n in zip(self.params, self.offsets, self.sizes):
            self.data[o:o + n].copy_(p.data.reshape(-1))
            p.data = self.data[o:o + n].view(p.shape)
            p.grad = self.grad[o:o + n].view(p.shape)
        # chunk tables
        beg, end, tens, t0 = [], [], [], [0]
        for ti, (o, n) in enumerate(zip(self.offsets, self.sizes)):
            for c in range(0, max(n, 1), CHUNK):
                beg.append(o + c)
                end.append(o + min(n, c + CHUNK))
                tens.append(ti)
            t0.append(len(beg))
        self.nchunks, self.ntensors = len(beg), len(self.params)
        self.chunk_beg = torch.tensor(beg, dtype=torch.int64, device=device)
        self.chunk_end = torch.tensor(end, dtype=torch.int64, device=device)
        self.chunk_tensor = torch.tensor(tens, dtype=torch.int32, device=device)
        self.tensor_chunk0 = torch.tensor(t0, dtype=torch.int32, device=device)

    def rebind(self):
        """Re-point param.data / param.grad at the arenas (after e.g. load_state_dict replaced them)."""
        for p, o, n in zip(self.params, self.offsets, self.sizes):
            if p.data.data_ptr() != self.data[o:o + n].data_ptr():
                self.data[o:o + n].copy_(p.data.reshape(-1))
                p.data = self.data[o:o + n].view(p.shape)
            if p.grad is None or p.grad.data_ptr() != self.grad[o:o + n].data_ptr():
                p.grad = self.grad[o:o + n].view(p.shape)

    def zero_grad(self):
        self.grad.zero_()


class LaProp(torch.optim.Optimizer):
    """Drop-in for utils/optim/laprop.py's LaProp (amsgrad/centered/weight_decay unsupported, as unused there),
    fused with clip_grad_agc_ and the LambdaLR warm-up of Dreamer (dreamer.py:209-225)."""

    def __init__(self, params, lr=4e-4, betas=(0.9, 0.999), eps=1e-15, agc=0.3, pmin=1e-3, warmup=0, arena=None,
                 ref_layouts=None, order=None):
        params = list(params)
        # per parameter: None, or (to_ref, from_ref) views between the internal and the reference layout, so that
        # state_dict() holds moments shaped like the reference's parameters (checkpoint interop)
        self.ref_layouts = list(ref_layouts) if ref_layouts is not None else [None] * len(params)
        # read into every gradient by the fused step: 1 / world after the data-parallel sum all-reduce, and
        # (tensor index, device scalar) gating one tensor (DreamerPro's prototype freeze); -1 = none
        self.grad_scale = 1.0
        self.gate = (-1, None)
        # the fused step zeroes every gradient it reads (sd_agc_laprop_step zero_grads): a graph-replayed update then
        # needs no zero_grad launch at its start
        self.zero_grads_after = False
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=0, amsgrad=False, centered=False))
        self.arena = arena if arena is not None else FlatArena(params, params[0].device, order)
        dev = self.arena.data.device
        self.exp_avg = torch.zeros_like(self.arena.data)
        self.exp_avg_sq = torch.zeros_like(self.arena.data)
        nb = nat.fns["sd_opt_scalars_bytes"]()
        self.scalars = torch.zeros((nb + 7) // 8, dtype=torch.float64, device=dev)  # step, lr_ema1, lr_ema2, lr
        self.workspace = torch.empty(3 * self.arena.nchunks, dtype=torch.float32, device=dev)
        self.grad_norms = torch.empty(self.arena.ntensors, dtype=torch.float32, device=dev)
        self.base_lr = float(lr)
        self.betas = (float(betas[0]), float(betas[1]))
        self.eps = float(eps)
        self.agc, self.pmin = float(agc), float(pmin)
        self.warmup = float(warmup or 0)
        self.host_steps = 0

    @torch.no_grad()
    def step(self, closure=None):
        self.launch_step()
        self.host_steps += 1

    @torch.no_grad()
    def launch_step(self):
        """Device part of step() (graph-capturable; host bookkeeping is in step())."""
        a = self.arena
        nat.call("sd_agc_laprop_step", K.p(a.data), K.p(a.grad), K.p(self.exp_avg), K.p(self.exp_avg_sq),
                 K.p(a.chunk_beg), K.p(a.chunk_end), K.p(a.chunk_tensor), K.p(a.tensor_chunk0), a.nchunks,
                 a.ntensors, K.p(self.workspace), K.p(self.scalars), K.p(self.grad_norms), self.agc, self.pmin,
                 self.base_lr, self.warmup, self.betas[0], self.betas[1], self.eps, float(self.grad_scale),
                 int(self.gate[0]), K.p(self.gate[1]), int(self.zero_grads_after), K.stream())

    def current_lr(self):
        """lr the NEXT step will use (LambdaLR semantics; host-side bookkeeping, no device sync)."""
        if self.warmup:
            return self.base_lr * min(1.0, (self.host_steps + 1) / self.warmup)
        return self.base_lr

    def zero_grad(self, set_to_none=False):
        self.arena.zero_grad()

    # ------------------------------------------------------------------ checkpoint compatibility
    def state_dict(self):
        sc = self.scalars.detach().cpu().tolist()
        steps = int(sc[0])
        st = {}
        a = self.arena
        for i, (o, n, p) in enumerate(zip(a.offsets, a.sizes, a.params)):
            if steps == 0:
                continue
            lay = self.ref_layouts[i]
            view = (lambda t: t) if lay is None else lay[0]
            st[i] = {"step": steps, "exp_avg": view(self.exp_avg[o:o + n].view(p.shape)).contiguous().clone(),
                     "exp_avg_lr_1": float(sc[1]), "exp_avg_lr_2": float(sc[2]),
                     "exp_avg_sq": view(self.exp_avg_sq[o:o + n].view(p.shape)).contiguous().clone()}
        lr = self.current_lr()
        groups = [{"lr": lr, "betas": self.betas, "eps": self.eps, "weight_decay": 0, "amsgrad": False,
                   "centered": False, "initial_lr": self.base_lr, "params": list(range(len(a.params)))}]
        return {"state": st, "param_groups": groups}

    def load_state_dict(self, sd, internal_layout=None):
        """internal_layout: None = infer each moment's layout from its shape (reference layout wins where both
        match, i.e. for square permutations), False = the file declares reference-layout moments (checkpoint.py
        writes `resume.moment_layout = "reference"`)."""
        a = self.arena
        st = sd.get("state", {})
        steps, e1, e2 = 0, 0.0, 0.0
        for i, (o, n) in enumerate(zip(a.offsets, a.sizes)):
            s = st.get(i, st.get(str(i)))
            if not s:
                continue
            lay, shape = self.ref_layouts[i], tuple(a.params[i].shape)
            ref_shape = shape if lay is None else tuple(lay[0](torch.empty(shape, device="meta")).shape)
            for dst, src in ((self.exp_avg, s["exp_avg"]), (self.exp_avg_sq, s["exp_avg_sq"])):
                # state_dict moments are in the reference layout (see state_dict); a tensor in the internal layout
                # (a file written before the moments were stored that way) is taken as it is only when its shape
                # cannot be mistaken for the reference one, anything else is an error rather than a silent broadcast
                if tuple(src.shape) == ref_shape:
                    src = src if lay is None else lay[1](src)
                elif tuple(src.shape) != shape or (internal_layout is False and lay is not None):
                    raise ValueError(f"LaProp state {i}: moment shape {tuple(src.shape)} matches neither the "
                                     f"reference layout {ref_shape} nor the internal layout {shape}")
                dst[o:o + n].view(shape).copy_(src)
            steps, e1, e2 = int(s["step"]), float(s["exp_avg_lr_1"]), float(s["exp_avg_lr_2"])
        self.scalars.copy_(torch.tensor([steps, e1, e2, 0.0][: self.scalars.numel()], dtype=torch.float64))
        self.host_steps = steps


class WarmupSchedule:
    """Stands in for LambdaLR(optimizer, min(1, (step+1)/warmup)) (dreamer.py:214-225); the warm-up itself is
    evaluated inside the fused optimiser kernel from the device step counter."""

    def __init__(self, optimizer):
        self.optimizer = optimizer

    def step(self):
        pass

    def get_lr(self):
        return [self.optimizer.current_lr()]

    def get_last_lr(self):
        return self.get_lr()
