"""Data-parallel decomposition on CPU (gloo, world_size 2): the exchange steps of sdreamer/parallel.py reproduce
the single-process results — gradient mean all-reduce, global ReturnEMA quantiles (all-gather), the sharded Barlow
loss/gradient (global column statistics + all-reduced cross-correlation), and global-row noise indexing of the
oracle (a 2-way row split of observe/imagine equals the full batch)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _TorchBarlowSteps:
    """torch restatement of parallel.BarlowSteps' HIP launches (csrc/misc.hip sd_barlow_*), same formulas, so the
    exchange decomposition runs on gloo CPU ranks; the HIP launches themselves are checked on the GPU
    (tests/test_gpu_ops.py test_barlow_dist_steps)."""

    @staticmethod
    def colsums(xd, x2):
        return torch.stack([xd.sum(0), x2.sum(0)])

    @staticmethod
    def center(xd, x2, sums, Nt):
        m = sums / Nt
        d1, d2 = xd - m[0], x2 - m[1]
        E = xd.shape[1]
        stats = torch.cat([(d1 * d1).sum(0), (d2 * d2).sum(0), (d1.t() @ d2).reshape(-1)])
        return d1, d2, stats

    @staticmethod
    def finish(stats, sums, Nt, d2):
        E = d2.shape[1]
        q, craw = stats[:2 * E].view(2, E), stats[2 * E:].view(E, E)
        s = torch.sqrt(q / (Nt - 1.0))
        sc = s + 1e-8
        c = craw / (sc[0][:, None] * sc[1][None, :]) / Nt
        return c, s, d2 / sc[1], (sums[1] - Nt * (sums[1] / Nt)) / sc[1]

    @staticmethod
    def loss(c, lambd):
        d = torch.diagonal(c)
        return (d - 1.0).pow(2).sum() + lambd * (c.pow(2).sum() - d.pow(2).sum())

    @staticmethod
    def grad_x1(x1, c, sums, st, n2, z2, g, lambd, Nt, world):
        eye = torch.eye(c.shape[0], dtype=torch.bool)
        dc = torch.where(eye, 2.0 * (c - 1.0), 2.0 * lambd * c) * g
        dn1 = n2 @ dc.t() / Nt
        sc = st[0] + 1e-8
        s0 = (dc @ z2) / Nt
        A = sc * (dc * c).sum(1)
        m1 = sums[0] / Nt
        return ((dn1 - s0 / Nt) / sc - (x1 - m1) * (A / (sc * sc * (Nt - 1) * st[0]))) * world


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from sdreamer import parallel
        parallel.BarlowSteps = _TorchBarlowSteps  # CPU ranks: torch stand-ins for the HIP launches (test only)
        torch.manual_seed(0)
        g = torch.randn(10)
        t = g * (rank + 1)
        parallel.allreduce_mean_(t)
        ok_ar = torch.allclose(t, g * 1.5)
        ret = torch.arange(6, dtype=torch.float32).view(3, 2) + 10 * rank
        allr = parallel.gather_returns(ret, world)
        ok_g = allr.shape == (6, 2) and float(allr[3, 0]) == 10.0
        # Barlow: full batch (64 rows) vs 2 shards of 32
        gen = torch.Generator().manual_seed(1)
        x1 = torch.randn(64, 16, generator=gen)
        x2 = torch.randn(64, 16, generator=gen)
        xs = x1[32 * rank: 32 * (rank + 1)].clone().requires_grad_()
        loss = parallel.barlow_dist(xs, x2[32 * rank: 32 * (rank + 1)], 5e-4, world)
        loss.backward()
        xr = x1.clone().requires_grad_()
        n1 = (xr - xr.mean(0)) / (xr.std(0) + 1e-8)
        n2 = (x2 - x2.mean(0)) / (x2.std(0) + 1e-8)
        c = n1.T @ n2 / 64
        off = ~torch.eye(16, dtype=torch.bool)
        ref = (torch.diagonal(c) - 1).pow(2).sum() + 5e-4 * c[off].pow(2).sum()
        ref.backward()
        ok_b = abs(float(loss) - float(ref)) < 1e-4 * abs(float(ref)) and torch.allclose(
            xs.grad / world, xr.grad[32 * rank: 32 * (rank + 1)], atol=1e-6, rtol=1e-4)  # x world: see _DistBarlowLoss
        q.put((rank, ok_ar, ok_g, ok_b))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_exchange_steps():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for rank, ok_ar, ok_g, ok_b in res:
        assert ok_ar and ok_g and ok_b, (rank, ok_ar, ok_g, ok_b)


def test_oracle_row_sharding_is_exact():
    """Noise is indexed by global row: observing / imagining two halves with row offsets == the full batch."""
    from golden_io import batch, initial, load_case
    from oracle.ref_cpu import Oracle
    z, cfg, spec, params, obs = load_case("proprio_dreamer")
    P = {k: torch.tensor(v) for k, v in params.items()}
    M = Oracle(spec, P)
    data = batch(z, 0, obs)
    init = initial(z, 0, spec)
    with torch.no_grad():
        emb = M.encode(data)
        full = M.observe(emb, data["action"], init, data["is_first"], 77)
        halves = [M.observe(emb[i:i + 2], data["action"][i:i + 2], (init[0][i:i + 2], init[1][i:i + 2]),
                            data["is_first"][i:i + 2], 77, row_offset=i) for i in (0, 2)]
        for j in range(3):
            assert torch.equal(torch.cat([h[j] for h in halves], 0), full[j])
        B, T = data["action"].shape[:2]
        start = (full[0].reshape(-1, spec.S, spec.K), full[1].reshape(-1, spec.D))
        f_full, a_full = M.imagine(start, 4, 5)
        n = B * T // 2
        f0, a0 = M.imagine((start[0][:n], start[1][:n]), 4, 5, row_offset=0)
        f1, a1 = M.imagine((start[0][n:], start[1][n:]), 4, 5, row_offset=n)
        assert torch.equal(torch.cat([f0, f1], 0), f_full) and torch.equal(torch.cat([a0, a1], 0), a_full)
