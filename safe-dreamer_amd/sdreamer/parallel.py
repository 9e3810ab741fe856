"""Data parallelism over the replay batch: one process per GPU, torch.distributed with the
"nccl" backend (= RCCL on ROCm, xGMI inside a node), gloo for CPU tests.

Exchange steps per update (every other stage is row-independent):
  1. gradient all-reduce (mean) of the flat fp32 gradient arena — one collective (sdreamer/optim.py);
  2. ReturnEMA: all-gather of the imagined λ-returns so every rank computes the same global quantiles
     (networks.py:417 takes the quantile over the whole batch);
  3. Barlow loss (r2dreamer): column sums / squared deviations and the E x E cross-correlation are all-reduced so
     the loss and its gradient equal the single-GPU values (dreamer.py:525-532 normalises over all B*T rows).
The noise is indexed by global row (oracle/noise.py), so an N-rank run reproduces the 1-rank batch exactly.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from . import kernels as K
from . import ops


def is_dist():
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def allreduce_mean_(t):
    if not is_dist():
        return t
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    t.mul_(1.0 / dist.get_world_size())
    return t


def gather_returns(ret, world):
    if world <= 1 or not is_dist():
        return ret
    out = [torch.empty_like(ret) for _ in range(dist.get_world_size())]
    dist.all_gather(out, ret.contiguous())
    return torch.cat(out, 0)


class DistBarlowFn(torch.autograd.Function):
    """Barlow loss over the GLOBAL batch with rows sharded across ranks (x1 local (n, E) with grad, x2 detached)."""

    @staticmethod
    def forward(ctx, x1, x2, lambd):
        x1, x2 = x1.contiguous(), x2.contiguous()
        n, E = x1.shape
        N = torch.tensor([float(n)], device=x1.device)
        dist.all_reduce(N)
        Nt = N.item()

        def stats(x):
            s = x.sum(0)
            dist.all_reduce(s)
            mu = s / Nt
            q = ((x - mu) ** 2).sum(0)
            dist.all_reduce(q)
            return mu, torch.sqrt(q / (Nt - 1))

        m1, s1 = stats(x1)
        m2, s2 = stats(x2)
        n1 = (x1 - m1) / (s1 + 1e-8)
        n2 = (x2 - m2) / (s2 + 1e-8)
        c = K.mm(n1.t().contiguous(), n2, alpha=1.0 / Nt)
        dist.all_reduce(c)
        eye = torch.eye(E, dtype=torch.bool, device=c.device)
        loss = (torch.diagonal(c) - 1.0).pow(2).sum() + lambd * c[~eye].pow(2).sum()
        ctx.save_for_backward(x1, m1, s1, n2, c)
        ctx.lambd, ctx.Nt = lambd, Nt
        return loss

    @staticmethod
    def backward(ctx, g):
        x1, m1, s1, n2, c = ctx.saved_tensors
        E = c.shape[0]
        eye = torch.eye(E, dtype=torch.bool, device=c.device)
        dc = torch.where(eye, 2.0 * (c - 1.0), 2.0 * ctx.lambd * c) * g
        dn1 = K.mm(n2, dc.t().contiguous(), alpha=1.0 / ctx.Nt)
        sc = s1 + 1e-8
        s0 = dn1.sum(0)
        dist.all_reduce(s0)
        A = (dn1 * (x1 - m1)).sum(0)
        dist.all_reduce(A)
        dx1 = (dn1 - s0 / ctx.Nt) / sc - (x1 - m1) * (A / (sc * sc * (ctx.Nt - 1) * s1))
        return dx1, None, None


def barlow(x1, x2, lambd, world):
    if world > 1 and is_dist():
        return DistBarlowFn.apply(x1, x2, lambd)
    return ops.BarlowFn.apply(x1, x2, lambd)
