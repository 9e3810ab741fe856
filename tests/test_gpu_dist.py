"""Data-parallel update on the GPU: 2 ranks (gloo, both on cuda:0) vs 1 rank on the full batch.

Each rank runs the product update on its half of the golden batch rows (row offset = rank * B/2, so it draws the
single-GPU noise of those rows) through the same code the 8-GPU bench runs: the two-stream schedule, eager warm-up
updates, then the captured phase graphs split at the exchange steps (Barlow statistics, the returns gather, the
gradient all-reduce — sdreamer/parallel.py). gloo stands in for RCCL (one GPU on the test box; RCCL refuses two
ranks on one device); the collectives are issued by the same calls (`parallel.collective`, and the bucketed gradient
all-reduce on the communication stream, Dreamer._allreduce_bucket). Stated tolerances:
world-model losses <= 1e-4 relative, other scalar losses <= 1e-3 (sums of differently ordered partial sums), the
parameters after 4 updates: L2 distance <= 2% of the L2 norm of the 4-update change, and <= 0.1% of the elements off
by more than 5% of the largest step (LaProp normalises per element, so summation-order noise on near-zero gradients
moves single elements by up to a step). The exchange steps themselves are held tighter: the all-reduced gradient
arena of update 0 (eager: the step leaves the gradients in place) matches the 1-rank gradients element-wise at the
golden gradient tolerance of test_cal_grad_matches_reference (2e-3 relative + 1e-4 of the tensor's largest |g|).
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
UPDATES = 4  # 2 eager + capture/replay + replay


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(name, rank, world, port, q):
    try:
        import torch
        import torch.distributed as dist
        from golden_io import batch, initial
        from test_gpu_dreamer import build_agent
        if world > 1:
            os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
            dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        ag, z, spec, obs = build_agent(name)
        ag.rank, ag.world = rank, world
        p0 = ag._optimizer.arena.data.detach().clone()
        data = batch(z, 0, obs, "cuda")
        init = initial(z, 0, spec, "cuda")
        B = data["action"].shape[0]
        b = B // world
        rows = slice(rank * b, (rank + 1) * b)
        data = {k: v[rows].contiguous() for k, v in data.items()}
        init = tuple(t[rows].contiguous() for t in init)
        losses = []
        g0 = None
        for u in range(UPDATES):
            _, mets = ag.update_batch(data, init, int(z["u0_seed"]) + u)
            losses.append({k: float(v) for k, v in mets.items() if k.startswith("loss/")})
            if u == 0:  # eager update: all-reduced (mean) gradients, left in the arena by the step
                g0 = ag._optimizer.arena.grad.detach().cpu().numpy().copy()
        torch.cuda.synchronize()
        p1 = ag._optimizer.arena.data.detach()
        a = ag._optimizer.arena
        spans = [(o, o + p.numel()) for o, p in zip(a.offsets, a.params)]
        q.put((rank, losses, (p1 - p0).cpu().numpy(), p1.cpu().numpy(), ag._graph is not None, g0, spans))
        if world > 1:
            dist.destroy_process_group()
    except BaseException as e:  # report instead of hanging the parent
        q.put((rank, repr(e), None, None, None, None, None))
        raise


def _run(name, world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(name, r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in procs:
        r = q.get(timeout=240)
        res[r[0]] = r
    for p in procs:
        p.join(timeout=60)
    for r in res.values():
        assert r[2] is not None, f"rank {r[0]} failed: {r[1]}"
    return res


@pytest.mark.parametrize("name", ["walker_r2", "walker_dreamer", "walker_infonce", "walker_r2aug", "walker_pro",
                                  "atari_r2", "maze_r2"])
def test_two_rank_update_equals_one_rank(name):
    one = _run(name, 1)[0]
    two = _run(name, 2)
    assert one[4] and two[0][4] and two[1][4], "the update was not graph-replayed"
    for u in range(UPDATES):
        for k, ref in one[1][u].items():
            # every loss is a mean over rows (equal shards: mean of the ranks' means); Barlow is global per rank
            got = [two[r][1][u][k] for r in (0, 1)]
            tol = 1e-4 if k[5:] in ("dyn", "rep", "rew", "con", "barlow", "image") else 1e-3
            assert abs(sum(got) / 2 - ref) <= tol * max(abs(ref), 1e-6), (u, k, got, ref)
            if k == "loss/barlow":
                assert abs(got[0] - got[1]) <= 1e-6 * abs(ref), (u, got)
    for rank in (0, 1):
        p_end = two[rank][3]
        d = p_end - one[3]
        rel_l2 = np.linalg.norm(d) / np.linalg.norm(one[2])
        frac = float((np.abs(d) > 0.05 * np.abs(one[2]).max()).mean())
        assert rel_l2 <= 0.02 and frac <= 1e-3, (rank, rel_l2, frac)
    assert np.array_equal(two[0][3], two[1][3]), "ranks diverged"
    # update 0's gradient arena after the exchange, element-wise per tensor, on both ranks
    bad = []
    for rank in (0, 1):
        g2 = two[rank][5]
        for lo, hi in one[6]:
            ref, got = one[5][lo:hi].astype(np.float64), g2[lo:hi].astype(np.float64)
            err = np.abs(got - ref) - (2e-3 * np.abs(ref) + 1e-4 * np.abs(ref).max() + 1e-12)
            if err.size and err.max() > 0:
                i = int(np.argmax(err))
                bad.append((rank, lo, hi, float(got[i]), float(ref[i])))
    assert not bad, bad[:8]
