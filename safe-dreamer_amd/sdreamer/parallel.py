"""Data parallelism over the replay batch: one process per GPU, torch.distributed with the
"nccl" backend (= RCCL on ROCm, xGMI inside a node), gloo for CPU tests.

Exchange steps per update (every other stage is row-independent):
  1. gradient all-reduce (mean) of the flat fp32 gradient arena — one collective (sdreamer/optim.py);
  2. ReturnEMA: the imagined λ-returns of every rank are all-gathered (rank order = global row order) so every rank
     computes the same global quantiles (networks.py:417 takes the quantile over the whole batch);
  3. InfoNCE (rep_loss=infonce): x2 of every rank is all-gathered (the negatives are the whole batch);
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


def all_gather_rows(x, world):
    """Every rank's rows of x stacked in rank order (the global batch's row order): one all-gather."""
    if world <= 1 or not is_dist():
        return x
    x = x.contiguous()
    out = torch.empty((world * x.shape[0],) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    collective(lambda: dist.all_gather_into_tensor(out, x))
    return out


def gather_returns(ret, world):
    """All ranks' returns stacked in rank order (the global batch's row order)."""
    return all_gather_rows(ret, world)


class BarlowSteps:
    """The per-rank arithmetic of the data-parallel Barlow loss as HIP launches (csrc/misc.hip sd_barlow_*, the two
    GEMMs on sd_gemm_f32); barlow_dist() puts the two all-reduces between them. tests/test_parallel_gloo.py swaps in
    a torch stand-in (CPU ranks) to check the decomposition; the GPU tests check each launch against torch fp32."""

    @staticmethod
    def colsums(xd, x2):
        sums = torch.empty(2, xd.shape[1], device=xd.device)
        K.colsum(xd, sums[0], accumulate=False)
        K.colsum(x2, sums[1], accumulate=False)
        return sums

    @staticmethod
    def center(xd, x2, sums, Nt):
        """-> d1, d2 and stats = [q (2, E) | d1^T d2 (E, E)] (this rank's sums)"""
        n, E = xd.shape
        d1, d2 = torch.empty_like(xd), torch.empty_like(x2)
        stats = torch.empty(2 * E + E * E, dtype=torch.float32, device=xd.device)
        K.nat.call("sd_barlow_center", K.p(xd), K.p(x2), K.p(sums), Nt, n, E, K.p(d1), K.p(d2), K.p(stats),
                   K.stream())
        K.gemm(d1.t(), d2, stats[2 * E:].view(E, E))
        return d1, d2, stats

    @staticmethod
    def finish(stats, sums, Nt, d2):
        """-> c (E, E), s (2, E) unbiased global stds, n2 = d2 / (s2 + 1e-8), z2 = global column sums of n2"""
        n, E = d2.shape
        dev = d2.device
        c, st = torch.empty(E, E, device=dev), torch.empty(2, E, device=dev)
        n2, z2 = torch.empty_like(d2), torch.empty(E, device=dev)
        K.nat.call("sd_barlow_finish", K.p(stats), K.p(sums), Nt, E, K.p(d2), n, K.p(c), K.p(st), K.p(n2), K.p(z2),
                   K.stream())
        return c, st, n2, z2

    @staticmethod
    def loss(c, lambd):
        E = c.shape[0]
        part = torch.empty(2 * 256, device=c.device)
        out = torch.empty(1, device=c.device)
        K.nat.call("sd_barlow_loss", K.p(c), E, float(lambd), K.p(part), 256, K.p(out), K.stream())
        return out[0]

    @staticmethod
    def grad_x1(x1, c, sums, st, n2, z2, g, lambd, Nt, world):
        R, E = x1.shape
        dc = torch.empty_like(c)
        K.nat.call("sd_barlow_dc", K.p(c), K.p(g.reshape(1).contiguous()), K.p(dc), E, float(lambd), K.stream())
        dn1 = K.mm(n2, dc.t(), alpha=1.0 / Nt)
        s0, A = torch.empty(E, device=c.device), torch.empty(E, device=c.device)
        K.nat.call("sd_barlow_rowstats", K.p(dc), K.p(c), K.p(z2), K.p(st[0]), float(Nt), E, K.p(s0), K.p(A),
                   K.stream())
        dx1 = torch.empty_like(x1)
        K.nat.call("sd_barlow_dist_dx", K.p(x1), K.p(dn1), K.p(sums), K.p(st[0]), K.p(s0), K.p(A), float(Nt),
                   float(world), R, E, K.p(dx1), K.stream())
        return dx1


class _DistBarlowLoss(torch.autograd.Function):
    """Barlow loss from the GLOBAL cross-correlation c, gradient w.r.t. this rank's rows of x1 (detached x2).

    With n = (x - m) / sc, sc = s + 1e-8, s the unbiased std over all Nt rows:
      dx1 = (dn1 - s0 / Nt) / sc - (x1 - m1) * A / (sc^2 (Nt - 1) s)
    where dn1 = n2 dc^T / Nt (local rows) and the two global row sums are
      s0_j = sum_r dn1[r, j] = sum_k dc[j, k] * z2_k / Nt     (z2 = global column sums of n2)
      A_j  = sum_r dn1[r, j] (x1[r, j] - m1[j]) = sc1_j * sum_k dc[j, k] c[j, k].
    Every rank holds the same global loss, so the true parameter gradient is the SUM of the ranks' partials; the
    arena all-reduce takes the MEAN (right for the per-row mean losses), so dx1 is scaled by world here."""

    @staticmethod
    def forward(ctx, x1, c, sums, st, n2, z2, lambd, Nt, world):
        ctx.save_for_backward(x1, c, sums, st, n2, z2)
        ctx.lambd, ctx.Nt, ctx.world = lambd, Nt, world
        return BarlowSteps.loss(c, lambd)

    @staticmethod
    def backward(ctx, g):
        x1, c, sums, st, n2, z2 = ctx.saved_tensors
        dx1 = BarlowSteps.grad_x1(x1, c, sums, st, n2, z2, g, ctx.lambd, ctx.Nt, ctx.world)
        return dx1, None, None, None, None, None, None, None, None


def barlow_dist(x1, x2, lambd, world):
    """R2-Dreamer Barlow loss (dreamer.py:525-532) over the global batch, rows sharded across ranks.
    x1 (n, E) with grad, x2 (n, E) detached; every rank holds the same n. Two all-reduces: the column sums, then the
    centred column sums of squares together with the centred cross-product d1^T d2 (E x E)."""
    x1c, x2 = x1.contiguous(), x2.detach().contiguous()
    n, E = x1c.shape
    Nt = float(n * world)
    xd = x1c.detach()
    sums = BarlowSteps.colsums(xd, x2)
    collective(lambda: dist.all_reduce(sums))
    _, d2, stats = BarlowSteps.center(xd, x2, sums, Nt)
    collective(lambda: dist.all_reduce(stats))
    c, st, n2, z2 = BarlowSteps.finish(stats, sums, Nt, d2)
    return _DistBarlowLoss.apply(x1c, c, sums, st, n2, z2, float(lambd), Nt, world)


def barlow(x1, x2, lambd, world):
    if world > 1 and is_dist():
        return barlow_dist(x1, x2, lambd, world)
    return ops.BarlowFn.apply(x1, x2, lambd)


def infonce(x1, x2, world):
    """InfoNCE (dreamer.py:533-542) with every rank's rows as negatives: x2 of all ranks is gathered (one
    all_gather_into_tensor, all_gather_rows), this rank's rows are labelled with their global column."""
    x2 = x2.detach().contiguous()
    if world > 1 and is_dist():
        x2g = all_gather_rows(x2, world)
        return ops.InfoNCEFn.apply(x1, x2g, dist.get_rank() * x2.shape[0])
    return ops.InfoNCEFn.apply(x1, x2, 0)