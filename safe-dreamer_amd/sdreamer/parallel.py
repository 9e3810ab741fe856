"""Data parallelism over the replay batch: one process per GPU, torch.distributed with the
"nccl" backend (= RCCL on ROCm, xGMI inside a node), gloo for CPU tests.

Exchange steps per update (every other stage is row-independent):
  1. gradient all-reduce (mean) of the flat fp32 gradient arena — one collective (sdreamer/optim.py);
  2. ReturnEMA: the imagined λ-returns of every rank are gathered (each rank writes its rows into a zeroed
     (world·N, H) buffer, one sum all-reduce) so every rank computes the same global quantiles
     (networks.py:417 takes the quantile over the whole batch);
  3. InfoNCE (rep_loss=infonce): x2 of every rank is gathered (the negatives are the whole batch);
  4. Barlow loss (r2dreamer): two all-reduces per update — column sums, then column sums of squared deviations
     together with the centred E x E cross-product — so loss and gradient equal the single-GPU values
     (dreamer.py:525-532 normalises over all B*T rows). The backward needs no exchange: the two batch sums the
     standardisation backward takes are functions of the global c and column sums (see _DistBarlowLoss).
The noise is indexed by global row (oracle/noise.py), so an N-rank run reproduces the 1-rank batch exactly.

Every exchange goes through `collective(fn)`. Eagerly it runs fn. While a stream phase is being captured by
`capture_phase`, it ends the current HIP graph there and records fn, so the phase replays as
graph, collective, graph, ... with the collective issued eagerly on the phase's stream (RCCL calls are never
captured into a graph).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from . import kernels as K
from . import ops


def is_dist():
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


# ------------------------------------------------------------------------------------------- graph segments
class PhaseGraph:
    """One stream phase as a chain of captured graphs and the collectives between them."""

    def __init__(self, error_mode):
        self.items = []
        self._mode = error_mode
        self._g = None

    def _begin(self):
        self._g = torch.cuda.CUDAGraph()
        self._g.capture_begin(capture_error_mode=self._mode)

    def _end(self):
        self._g.capture_end()
        self.items.append(self._g)
        self._g = None

    def _split(self, fn):
        self._end()
        self.items.append(fn)
        self._begin()

    def first_collective(self):
        """Index of the first collective (len(items) if none): replay(0, k) runs the part before it."""
        for i, it in enumerate(self.items):
            if not isinstance(it, torch.cuda.CUDAGraph):
                return i
        return len(self.items)

    @property
    def n_collectives(self):
        return sum(not isinstance(it, torch.cuda.CUDAGraph) for it in self.items)

    def replay(self, lo=0, hi=None):
        for it in self.items[lo:hi]:
            if isinstance(it, torch.cuda.CUDAGraph):
                it.replay()
            else:
                it()


_active = None


def capture_phase(fn, stream, error_mode="global"):
    """Capture fn() on `stream` as a PhaseGraph (split at every `collective`). Returns (phase, fn's result)."""
    global _active
    if _active is not None:
        raise RuntimeError("nested phase capture")
    pg = PhaseGraph(error_mode)
    torch.cuda.synchronize()
    with torch.cuda.stream(stream):
        pg._begin()
        _active = pg
        try:
            out = fn()
        except BaseException:
            _active = None
            pg._g.capture_end()
            raise
        _active = None
        pg._end()
    return pg, out


def collective(fn):
    """Run an exchange step now (eager) or record it as a split point of the phase being captured."""
    if _active is None:
        fn()
    else:
        _active._split(fn)


# ------------------------------------------------------------------------------------------- exchange steps
def allreduce_mean_(t):
    if not is_dist():
        return t
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    t.mul_(1.0 / dist.get_world_size())
    return t


def gather_returns(ret, world):
    """All ranks' returns stacked in rank order (the global batch's row order)."""
    if world <= 1 or not is_dist():
        return ret
    n = ret.shape[0]
    rank = dist.get_rank()
    out = torch.zeros((world * n,) + tuple(ret.shape[1:]), dtype=ret.dtype, device=ret.device)
    out[rank * n:(rank + 1) * n].copy_(ret)
    collective(lambda: dist.all_reduce(out))
    return out


class _DistBarlowLoss(torch.autograd.Function):
    """Barlow loss from the GLOBAL cross-correlation c, gradient w.r.t. this rank's rows of x1 (detached x2).

    With n = (x - m) / sc, sc = s + 1e-8, s the unbiased std over all Nt rows:
      dx1 = (dn1 - s0 / Nt) / sc - (x1 - m1) * A / (sc^2 (Nt - 1) s)
    where dn1 = n2 dc^T / Nt (local rows) and the two global row sums are
      s0_j = sum_r dn1[r, j] = sum_k dc[j, k] * z2_k / Nt     (z2 = global column sums of n2)
      A_j  = sum_r dn1[r, j] (x1[r, j] - m1[j]) = sc1_j * sum_k dc[j, k] c[j, k].
    Every rank holds the same global loss, so the true parameter gradient is the SUM of the ranks' partials; the
    arena all-reduce takes the MEAN (right for the per-row mean losses), so dx1 is scaled by world here.
    """

    @staticmethod
    def forward(ctx, x1, c, m1, s1, n2, z2, lambd, Nt, world):
        d = torch.diagonal(c)
        loss = (d - 1.0).pow(2).sum() + lambd * (c.pow(2).sum() - d.pow(2).sum())
        ctx.save_for_backward(x1, c, m1, s1, n2, z2)
        ctx.lambd, ctx.Nt, ctx.world = lambd, Nt, world
        return loss

    @staticmethod
    def backward(ctx, g):
        x1, c, m1, s1, n2, z2 = ctx.saved_tensors
        lambd, Nt = ctx.lambd, ctx.Nt
        eye = torch.eye(c.shape[0], dtype=torch.bool, device=c.device)
        dc = torch.where(eye, 2.0 * (c - 1.0), 2.0 * lambd * c) * g
        dn1 = K.mm(n2, dc.t().contiguous(), alpha=1.0 / Nt)
        sc = s1 + 1e-8
        s0 = (dc @ z2) / Nt
        A = sc * (dc * c).sum(1)
        dx1 = (dn1 - s0 / Nt) / sc - (x1 - m1) * (A / (sc * sc * (Nt - 1) * s1))
        return dx1 * ctx.world, None, None, None, None, None, None, None, None


def barlow_dist(x1, x2, lambd, world):
    """R2-Dreamer Barlow loss (dreamer.py:525-532) over the global batch, rows sharded across ranks.
    x1 (n, E) with grad, x2 (n, E) detached; every rank holds the same n."""
    x1c, x2 = x1.contiguous(), x2.detach().contiguous()
    n, E = x1c.shape
    Nt = float(n * world)
    xd = x1c.detach()
    sums = torch.stack([xd.sum(0), x2.sum(0)])  # (2, E)
    collective(lambda: dist.all_reduce(sums))
    m = sums / Nt
    d1, d2 = xd - m[0], x2 - m[1]
    stats = torch.empty(2 * E + E * E, dtype=torch.float32, device=x1.device)
    q, craw = stats[:2 * E].view(2, E), stats[2 * E:].view(E, E)
    torch.sum(d1 * d1, 0, out=q[0])
    torch.sum(d2 * d2, 0, out=q[1])
    craw.copy_(K.mm(d1.t(), d2))
    collective(lambda: dist.all_reduce(stats))
    s = torch.sqrt(q / (Nt - 1.0))
    sc = s + 1e-8
    c = craw / (sc[0][:, None] * sc[1][None, :]) / Nt
    n2 = d2 / sc[1]
    z2 = (sums[1] - Nt * m[1]) / sc[1]
    return _DistBarlowLoss.apply(x1c, c, m[0], s[0], n2, z2, float(lambd), Nt, world)


def barlow(x1, x2, lambd, world):
    if world > 1 and is_dist():
        return barlow_dist(x1, x2, lambd, world)
    return ops.BarlowFn.apply(x1, x2, lambd)


def infonce(x1, x2, world):
    """InfoNCE (dreamer.py:533-542) with every rank's rows as negatives: x2 of all ranks is gathered (one sum
    all-reduce of a zero-padded buffer), this rank's rows are labelled with their global column."""
    x2 = x2.detach().contiguous()
    if world > 1 and is_dist():
        n = x2.shape[0]
        rank = dist.get_rank()
        x2g = torch.zeros((world * n,) + tuple(x2.shape[1:]), dtype=x2.dtype, device=x2.device)
        x2g[rank * n:(rank + 1) * n].copy_(x2)
        collective(lambda: dist.all_reduce(x2g))
        return ops.InfoNCEFn.apply(x1, x2g, rank * n)
    return ops.InfoNCEFn.apply(x1, x2, 0)