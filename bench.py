#!/usr/bin/env python
"""Headline benchmark: imagined latent steps / s of the full Dreamer update (BASELINE.json `metric`).

Workload (BASELINE.json configs[1]): DMC-vision walker_walk 64x64x3, rep_loss=r2dreamer, B16 L64 H15 per GPU,
synthetic data (uniform uint8 images, U(-1,1) actions, U(0,1) rewards), reference-initialised
random weights. One step = one `Dreamer.update(replay_buffer)` (dreamer.py:402-451): on-device replay sampling,
encoder + RSSM observe scan fwd/bwd, prior/KL, Barlow, heads, H+1-step imagination, λ-returns, ReturnEMA,
actor/critic/replay-value losses, backward, (all-reduce), AGC + LaProp. Each step consumes B*L*H imagined latents.

Run: python bench.py [--gpus N --steps K --warmup W]; N > 1 under torch.distributed.run (weak scaling: B=16/GPU,
gradient all-reduce over RCCL). Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "safe-dreamer_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "imagined latent steps/sec at B16\u00b7L64\u00b7H15, 1/2/4/8 MI355X; WM-loss \u0394 vs ref"  # BASELINE.json
PEAK_FP32_MFMA = 157.3  # TFLOP/s, MI355X_MICROARCH.md (dense f32 matrix = f32 vector peak)
PEAK_HBM = 8000.0  # GB/s spec


class _Sp:
    def __init__(self, shape):
        self.shape = tuple(shape)


class _Spaces:
    def __init__(self, d):
        self.spaces = d


def synth_buffer(cfg, device, rank, T=160, A=6):
    """Fill an HBM replay buffer with synthetic walker-like transitions (16 envs x T steps, one episode each)."""
    from sdreamer.buffer import Buffer
    g = torch.Generator(device="cpu").manual_seed(1000 + rank)
    E = 16
    S, Kd, D = int(cfg.model.rssm.stoch), int(cfg.model.rssm.discrete), int(cfg.model.rssm.deter)
    buf = Buffer(cfg.buffer, device=device, seed=rank)
    first = torch.zeros(T, E, 1, dtype=torch.bool)
    first[0] = True
    idx = torch.randint(0, Kd, (T, E, S), generator=g)
    data = {
        "image": torch.randint(0, 256, (T, E, 64, 64, 3), dtype=torch.uint8, generator=g),
        "action": torch.rand(T, E, A, generator=g) * 2 - 1,
        "reward": torch.rand(T, E, 1, generator=g),
        "is_first": first,
        "is_last": torch.zeros(T, E, 1, dtype=torch.bool),
        "is_terminal": torch.zeros(T, E, 1, dtype=torch.bool),
        "episode": torch.arange(E, dtype=torch.int32)[None].expand(T, E).contiguous(),
        "stoch": torch.nn.functional.one_hot(idx, Kd).float(),
        "deter": torch.zeros(T, E, D),
    }
    buf.add_sequence({k: v.to(device) for k, v in data.items()})
    return buf


def cpu_baseline(cfg, n_updates, threads):
    """The CPU oracle (oracle/ref_cpu.py: fp32 restatement of the reference update) on the host cores."""
    from oracle.init import params_for
    from oracle.ref_cpu import OracleAgent, Spec
    torch.set_num_threads(threads)
    B, L = int(cfg.batch_size), int(cfg.batch_length)
    spec = Spec(cfg.model, {"image": (64, 64, 3)}, 6, False)
    ag = OracleAgent(spec, params_for(spec.shapes, 0))
    g = torch.Generator().manual_seed(0)
    first = torch.zeros(B, L, 1, dtype=torch.bool)
    first[:, 0] = True
    data = {"image": torch.randint(0, 256, (B, L, 64, 64, 3), generator=g, dtype=torch.uint8).float() / 255.0,
            "action": torch.rand(B, L, 6, generator=g) * 2 - 1, "reward": torch.rand(B, L, 1, generator=g),
            "is_first": first, "is_last": torch.zeros(B, L, 1, dtype=torch.bool),
            "is_terminal": torch.zeros(B, L, 1, dtype=torch.bool)}
    init = (torch.zeros(B, spec.S, spec.K), torch.zeros(B, spec.D))
    times = []
    for i in range(n_updates + 1):
        t0 = time.perf_counter()
        ag.update(data, init, seed=i)
        if i:
            times.append(time.perf_counter() - t0)
    return statistics.median(times)


def dominant_probe(K):
    """Roofline probe on the dominant kernel of the step: the encoder's second stage forward, conv + MaxPool2d(2) +
    RMSNorm2D + SiLU in one launch (implicit GEMM, M = B*L*32*32 pixels, N = 48, K = 5*5*32), the largest MFMA launch
    of the update. Algorithmic work = 2*M*N*K FLOP per launch."""
    if not K.ops_fused_pool():
        def flops(a):  # sd_conv2d_fwd(in, w, b, out, Nb, Hs, Ws, Ci, Co, kh, kw, pad, ups, stream)
            Nb, Hs, Ws, Ci, Co, kh, kw, ups = a[4], a[5], a[6], a[7], a[8], a[9], a[10], a[12]
            return 2.0 * Nb * (Hs << ups) * (Ws << ups) * Co * kh * kw * Ci
        return K.LaunchProbe("sd_conv2d_fwd", lambda a: a[7] == 32 and a[8] == 48 and a[12] == 0, flops,
                             label="conv_fwd16<48> (encoder conv2: 32->48 ch, 32x32, 5x5; implicit GEMM, "
                                   "v_mfma_f32_16x16x4_f32, N tile = 48 channels)")

    def flops(a):  # sd_conv2d_fwd_pool(in, w, b, nw, pooled, amax, y, rstd, Nb, Hs, Ws, Ci, Co, kh, kw, ...)
        Nb, Hs, Ws, Ci, Co, kh, kw = a[8], a[9], a[10], a[11], a[12], a[13], a[14]
        return 2.0 * Nb * Hs * Ws * Co * kh * kw * Ci
    return K.LaunchProbe("sd_conv2d_fwd_pool", lambda a: a[11] == 32 and a[12] == 48, flops,
                         label="conv_fwd16_pool<48> (encoder stage 2: 32->48 ch, 32x32, 5x5 conv + 2x2 max-pool + "
                               "RMSNorm + SiLU epilogue; implicit GEMM, v_mfma_f32_16x16x4_f32, N tile = 48)")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="dmc/cnn")
    ap.add_argument("--cpu-updates", type=int, default=3)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-roofline", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=device)

    from sdreamer import kernels as K
    from sdreamer.config import load_config
    from sdreamer.dreamer import Dreamer

    cfg = load_config(args.config, [f"device=cuda:{local}", "model.compile=False"])
    B, L, H = int(cfg.batch_size), int(cfg.batch_length), int(cfg.model.imag_horizon)
    torch.manual_seed(0)  # identical initial weights on every rank
    agent = Dreamer(cfg.model, _Spaces({"image": _Sp((64, 64, 3))}), _Sp((6,)), rank=rank, world=world)
    buf = synth_buffer(cfg, device, rank)

    # roofline probe on the dominant kernel: sees its launch (eager warm-up or graph capture), then re-times that
    # exact launch with HIP events on its stream after the timed steps
    probe = None if args.no_roofline else dominant_probe(K)
    for _ in range(args.warmup):
        agent.update(buf)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        agent.update(buf)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if probe is not None:
        probe.stop()
        probe.replay(20)
    if world > 1:
        t = torch.tensor([dt], device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = t.item()
    ms = dt / args.steps * 1000.0
    value = world * B * L * H * args.steps / dt

    out = {
        "metric": METRIC,
        "value": value, "unit": "imagined_latents/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": ms, "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic (uniform uint8 64x64x3 images, U(-1,1) actions, U(0,1) rewards; random-init weights)",
        "config": {"workload": "dmc walker_walk vision, rep_loss=r2dreamer, per-GPU B16 L64 H15 (BASELINE configs[1])",
                   "global_batch": B * world, "seq_len": L, "imag_horizon": H, "parallelism": f"dp{world}"},
    }
    if probe is not None:
        out["roofline"] = probe.report()
        # HBM bytes per launch of the same kernel from separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes
        # (tools/roofline_traffic.py: gfx950 FETCH_SIZE x2 correction), committed under profiles/
        tf = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "r01_roofline_traffic.json")
        if os.path.exists(tf):
            t = json.load(open(tf))
            if out["roofline"] and out["roofline"]["kernel"].startswith(t.get("kernel", "?") + " ") \
                    and t.get("traffic_bytes"):
                out["roofline"]["traffic"] = t["traffic_bytes"]
                out["roofline"]["traffic_source"] = "profiles/r01_roofline_traffic.json (rocprofv3 --pmc)"
                out["roofline"]["algorithmic_bytes"] = t.get("algorithmic_bytes")
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        threads = min(len(os.sched_getaffinity(0)), 16)
        cfg_cpu = load_config(args.config, ["device=cpu", "model.compile=False"])
        t_cpu = cpu_baseline(cfg_cpu, args.cpu_updates, threads)
        out["cpu_baseline"] = {"value": B * L * H / t_cpu, "unit": "imagined_latents/s", "cores": threads,
                               "kind": "port", "cpu": platform.processor() or platform.machine(),
                               "sample": f"oracle/ref_cpu.py OracleAgent.update() at walker B{B} L{L} H{H} fp32, "
                                         f"median of {args.cpu_updates} after 1 warm-up ({t_cpu:.2f} s/update)"}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
