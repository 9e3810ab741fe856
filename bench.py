#!/usr/bin/env python
"""Headline benchmark: imagined latent steps / s of the full Dreamer update (BASELINE.json `metric`).

Workload (default, BASELINE.json configs[1]): DMC-vision walker_walk 64x64x3, rep_loss=r2dreamer, B16 L64 H15 per
GPU; --config selects another BASELINE workload (WORKLOADS), --global-batch splits its batch over the ranks;
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


# --config -> the BASELINE.json workload it is (act dim, one-hot actions, label). Weak scaling keeps the config's
# batch per GPU; --global-batch divides it over the ranks instead (configs[2]: B64 over 8 GPUs = 8 rows per GPU).
WORKLOADS = {
    "dmc/cnn": (6, False, "dmc walker_walk vision 64x64x3, rep_loss=r2dreamer (BASELINE configs[1])"),
    "dmc/walker_dreamer": (6, False, "dmc walker_walk vision 64x64x3, rep_loss=dreamer conv decoder (BASELINE configs[2])"),
    "dmc/atari_breakout": (4, True, "Atari100k-like breakout 64x64x3, 4 one-hot actions, 32x32 stoch, r2dreamer "
                                    "(BASELINE configs[3], synthetic)"),
    "dmc/memory_maze": (6, True, "Memory-Maze-like 9x9 64x64x3, 6 one-hot actions, deter 4096, r2dreamer "
                                 "(BASELINE configs[4], synthetic)"),
}
# fwd+bwd matmul/conv FLOP of one update at the headline workload (FlopCounterMode on the reference)
UPDATE_FLOP = {("dmc/cnn", 16, 64, 15): 927.7e9}


def synth_buffer(cfg, device, rank, T=160, A=6, discrete=False):
    """Fill an HBM replay buffer with synthetic transitions (16 envs x T steps, one episode each): uniform uint8
    images, U(-1,1) actions (one-hot of a uniform index for discrete action spaces), U(0,1) rewards."""
    from sdreamer.buffer import Buffer
    g = torch.Generator(device="cpu").manual_seed(1000 + rank)
    E = 16
    S, Kd, D = int(cfg.model.rssm.stoch), int(cfg.model.rssm.discrete), int(cfg.model.rssm.deter)
    buf = Buffer(cfg.buffer, device=device, seed=rank)
    first = torch.zeros(T, E, 1, dtype=torch.bool)
    first[0] = True
    idx = torch.randint(0, Kd, (T, E, S), generator=g)
    if discrete:
        act = torch.nn.functional.one_hot(torch.randint(0, A, (T, E), generator=g), A).float()
    else:
        act = torch.rand(T, E, A, generator=g) * 2 - 1
    data = {
        "image": torch.randint(0, 256, (T, E, 64, 64, 3), dtype=torch.uint8, generator=g),
        "action": act,
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


def trace_mark(tag):
    """an empty dispatch a rocprofv3 kernel trace can find (sd_trace_mark): tags 1 / 2 bracket the timed steps"""
    from sdreamer import _native as nat
    from sdreamer import kernels as K
    nat.call("sd_trace_mark", int(tag), K.stream())


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or platform.machine()


def cpu_baseline(cfg, n_updates, threads, A=6, discrete=False):
    """The CPU oracle (oracle/ref_cpu.py: fp32 restatement of the reference update) on the host cores."""
    from oracle.init import params_for
    from oracle.ref_cpu import OracleAgent, Spec
    torch.set_num_threads(threads)
    B, L = int(cfg.batch_size), int(cfg.batch_length)
    spec = Spec(cfg.model, {"image": (64, 64, 3)}, A, discrete)
    ag = OracleAgent(spec, params_for(spec.shapes, 0))
    g = torch.Generator().manual_seed(0)
    first = torch.zeros(B, L, 1, dtype=torch.bool)
    first[:, 0] = True
    act = torch.nn.functional.one_hot(torch.randint(0, A, (B, L), generator=g), A).float() if discrete else \
        torch.rand(B, L, A, generator=g) * 2 - 1
    data = {"image": torch.randint(0, 256, (B, L, 64, 64, 3), generator=g, dtype=torch.uint8).float() / 255.0,
            "action": act, "reward": torch.rand(B, L, 1, generator=g),
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


def wm_loss_parity():
    """'WM-loss Δ vs ref' (BASELINE.json metric): the product's first update on the walker r2dreamer golden case —
    the reference's own update() outputs, generated by tests/golden/gen_golden.py — with the reference weights, batch,
    initial latents and noise seed. Returns the max relative error over the world-model loss terms and the terms."""
    import copy
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from golden_io import CASES, batch, initial, load_case
    from sdreamer.config import load_config
    from sdreamer.dreamer import Dreamer
    name = "walker_r2"
    z, _, spec, params, obs = load_case(name)
    gcfg = load_config(CASES[name][0], ["device=cuda:0", "model.compile=False", f"model.imag_horizon={int(z['meta_H'])}"])
    ag = Dreamer(copy.deepcopy(gcfg.model), _Spaces({k: _Sp(v) for k, v in obs.items()}), _Sp((int(z["meta_A"]),)))
    sd = {k: torch.from_numpy(v) for k, v in params.items()}
    for k, sk in spec.slow_names.items():
        sd[sk] = torch.from_numpy(params[k])
    sd["return_ema.ema_vals"] = torch.zeros(2)
    ag.load_state_dict(sd, strict=False)
    data = batch(z, 0, obs, "cuda")
    data["image"] = torch.from_numpy(z["u0_in_image"]).cuda()
    _, mets = ag.update_batch(data, initial(z, 0, spec, "cuda"), int(z["u0_seed"]))
    terms = {}
    for k in ("dyn", "rep", "rew", "con", "barlow"):
        ref = float(z[f"u0_m_loss/{k}"])
        terms[k] = abs(float(mets[f"loss/{k}"]) - ref) / max(abs(ref), 1e-6)
    scales = {k: float(ag._loss_scales[k]) for k in terms}  # WM total = sum of scaled WM terms, SURVEY §8(d)
    wm = sum(scales[k] * float(mets[f"loss/{k}"]) for k in scales)
    wm_ref = sum(scales[k] * float(z[f"u0_m_loss/{k}"]) for k in scales)
    return {"wm_loss_rel_err": abs(wm - wm_ref) / abs(wm_ref), "max_term_rel_err": max(terms.values()),
            "terms": terms, "case": f"tests/golden/{name}.npz (reference update() outputs, "
                                    f"B{int(z['meta_B'])} L{int(z['meta_T'])} H{int(z['meta_H'])})"}


def wm_loss_parity_full(name="C2_walker_r2"):
    """'WM-loss Δ vs ref' at the benched size: one product update at B16 L64 H15 (walker r2dreamer, BASELINE configs[1])
    against the REAL reference's update() on the same weights, batch, initial latents and noise seed —
    tests/golden/full_C2_walker_r2.npz, written in the build container by tests/golden/gen_golden.py `full` (the
    inputs are regenerated from the case name by tests/fullsize_io.py). Checker leg, run beside the CPU baseline:
    the weights come from the parity-fixture generator oracle/init.py. Returns the relative error of the scaled WM
    total and of each world-model term, and the posterior indices that differ from the reference's."""
    import copy
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from fullsize_io import FULL, OVERRIDES, PARAM_SEED, SEED, fixture_path, full_inputs, load_fixture
    from oracle.init import params_for
    from oracle.ref_cpu import Spec
    from sdreamer.config import load_config
    from sdreamer.dreamer import Dreamer
    cfg_name, ovr, obs, A, discrete, B, L, H = FULL[name]
    z = load_fixture(name)
    ccfg = load_config(cfg_name, ["device=cpu"] + ovr + OVERRIDES)
    spec = Spec(ccfg.model, obs, A, discrete)
    params = params_for(spec.shapes, PARAM_SEED)
    data_np, init_np = full_inputs(name, spec.K, spec.S, spec.D)
    gcfg = load_config(cfg_name, ["device=cuda:0"] + ovr + OVERRIDES)
    ag = Dreamer(copy.deepcopy(gcfg.model), _Spaces({k: _Sp(v) for k, v in obs.items()}), _Sp((A,)))
    sd = {k: torch.from_numpy(v) for k, v in params.items()}
    for k, sk in spec.slow_names.items():
        sd[sk] = torch.from_numpy(params[k])
    sd["return_ema.ema_vals"] = torch.zeros(2)
    ag.load_state_dict(sd, strict=False)
    (ps, _), mets = ag.update_batch({k: torch.from_numpy(v).cuda() for k, v in data_np.items()},
                                    tuple(torch.from_numpy(v).cuda() for v in init_np), SEED)
    torch.cuda.synchronize()
    keys = [k for k in ("dyn", "rep", "rew", "con", "barlow") if f"m_loss/{k}" in z]
    terms = {k: abs(float(mets[f"loss/{k}"]) - float(z[f"m_loss/{k}"])) / max(abs(float(z[f"m_loss/{k}"])), 1e-6)
             for k in keys}
    sc = {k: float(ag._loss_scales[k]) for k in keys}
    wm = sum(sc[k] * float(mets[f"loss/{k}"]) for k in keys)
    wm_ref = sum(sc[k] * float(z[f"m_loss/{k}"]) for k in keys)
    flips = int((ps.argmax(-1).cpu().numpy() != z["post_idx"]).sum())
    return {"wm_loss_rel_err": abs(wm - wm_ref) / abs(wm_ref), "max_term_rel_err": max(terms.values()),
            "terms": terms, "posterior_index_mismatches": flips, "posterior_indices": int(z["post_idx"].size),
            "case": f"{os.path.relpath(fixture_path(name), ROOT)} (the reference's own update() outputs at "
                    f"B{B} L{L} H{H}, same weights / batch / noise seed)"}


IMAG_KERNELS = {  # sd_imagine_step_kernel `which` -> (label, FLOP per launch as f(N, D, U, Dg))
    0: ("k_lin<32, 32> x3 (imagination step: img_net_0 + _dyn_in0 + actor layer 0's deter part, three (N, D) x (D, U) "
        "GEMMs in one launch, RMSNorm row partials in the epilogue; v_mfma_f32_16x16x4_f32)",
        lambda N, D, U, Dg: 3 * 2.0 * N * D * U),
    1: ("k_hid (imagination step: _dyn_hid BlockLinear, K = Dg + 3U per block, RMSNorm + SiLU of x0 / x1 in the A "
        "loader; bf16x6)", lambda N, D, U, Dg: 2.0 * N * D * (Dg + 3 * U)),
    2: ("k_gate (imagination step: _dyn_gru BlockLinear + GRU epilogue, RMSNorm + SiLU of hp in the A loader; bf16x6)",
        lambda N, D, U, Dg: 2.0 * N * 3 * D * Dg),
}


def imag_kernel_probe(agent, cfg, which=0, reps=30):
    """Roofline probe on the update's dominant kernel symbol, k_lin<32, 32> (imagination; largest total time per
    update, profiles/r02_kernel_summary.md): the imagination runs once at the update's shape (N = B*L start rows),
    then its step-t launch is re-issued alone (sd_imagine_step_kernel: same descriptor, workspace and grid) `reps`
    times over t = 0 .. H-1, back to back between two HIP events on the stream it is launched on (per-launch event
    pairs would add the event records' own cost to every launch; back to back only the ~1 us dispatch gap remains)."""
    import ctypes
    from sdreamer import _native as nat
    from sdreamer import kernels as K
    r = agent.rssm
    B, L, H = int(cfg.batch_size), int(cfg.batch_length), int(cfg.model.imag_horizon)
    N, H1, dev = B * L, H + 1, agent.device
    SK, D, U, G = r.flat_stoch, r._deter, r._hidden, r._blocks
    g = torch.Generator(device=dev).manual_seed(11)
    idx = torch.randint(0, r._discrete, (N, r._stoch), device=dev, generator=g)
    feats = torch.empty(H1, N, SK + D, device=dev)
    actions = torch.empty(H1, N, agent.act_dim, device=dev)
    feats[0, :, :SK] = torch.nn.functional.one_hot(idx, r._discrete).float().reshape(N, SK)
    feats[0, :, SK:] = torch.randn(N, D, device=dev, generator=g)
    keep = {}
    with torch.no_grad():
        agent._imagine_fused(feats, actions, H1, 5, 0, keep=keep)
    torch.cuda.synchronize()
    desc = keep["desc"]
    label, flop = IMAG_KERNELS[which]
    work = flop(N, D, U, D // G)
    nat.call("sd_imagine_step_kernel", ctypes.addressof(desc), which, 0, K.stream())  # warm
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for i in range(reps):
        nat.call("sd_imagine_step_kernel", ctypes.addressof(desc), which, i % H, K.stream())
    e.record()
    torch.cuda.synchronize()
    avg_ms = s.elapsed_time(e) / reps
    achieved = work / (avg_ms * 1e-3) / 1e12
    return {"bound": "mfma", "achieved": achieved, "peak": PEAK_FP32_MFMA, "unit": "TFLOP/s",
            "frac": achieved / PEAK_FP32_MFMA, "key": ("k_lin", "k_hid", "k_gate")[which], "kernel": label,
            "launches": reps, "avg_us": avg_ms * 1e3,
            "work_per_launch": work, "shape": f"N={N} D={D} U={U}"}


def dominant_probe(K):
    """Secondary roofline probe: the encoder's second stage forward, conv + MaxPool2d(2) + RMSNorm2D + SiLU in one
    launch (direct conv, M = B*L*32*32 pixels, N = 48, K = 5*5*32), the largest single MFMA launch of the update
    (DESIGN.md §5). Algorithmic work = 2*M*N*K FLOP per launch."""
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
                         label="conv_fwd_direct_pool<48> (encoder stage 2: 32->48 ch, 32x32, 5x5 conv + 2x2 max-pool + "
                               "RMSNorm + SiLU epilogue; direct conv from an LDS input patch, v_mfma_f32_16x16x4_f32, "
                               "N tile = 48)")


def phase_rooflines(agent, cfg, cfg_name, ms_update, reps=10):
    """SURVEY §8(d) 'report separately': (i) the imagination rollout alone (secondary metric N*H / t_rollout; FLOP =
    2 * weights per img_step (Deter + img_net) per imagined latent + 2 * actor weights per actor sample, H img_steps
    and H+1 actor samples per start row), (ii) the observe scan forward (RSSM.observe: bytes = the Deter + obs_net
    weights streamed once per step, the 'HBM GB/s on the recurrent scan' figure), (iv) the whole update (927.7
    GFLOP fwd+bwd at the headline config, SURVEY §8(d), FlopCounterMode on the reference; omitted for other
    workloads, whose update FLOP were not counted). Each phase runs eagerly after the
    timed steps on synthetic inputs of the update's shapes, bracketed by HIP events on the stream it launches on."""
    r = agent.rssm
    B, L, H = int(cfg.batch_size), int(cfg.batch_length), int(cfg.model.imag_horizon)
    N, dev = B * L, agent.device

    def numel(mod):
        return sum(p.numel() for p in mod.parameters())

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            fn()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / reps

    g = torch.Generator(device=dev).manual_seed(7)
    idx = torch.randint(0, r._discrete, (N, r._stoch), device=dev, generator=g)
    stoch = torch.nn.functional.one_hot(idx, r._discrete).float()
    deter = torch.randn(N, r._deter, device=dev, generator=g)
    with torch.no_grad():
        ms_img = timed(lambda: agent._imagine_tm((stoch, deter), H + 1, 3))
    p_step, p_act = numel(r._deter_net) + numel(r._img_net), numel(agent.actor)
    f_img = 2.0 * N * (H * p_step + (H + 1) * p_act)

    embed = torch.randn(B, L, r.embed_size, device=dev, generator=g)
    action = torch.rand(B, L, r._act_dim, device=dev, generator=g) * 2 - 1
    reset = torch.zeros(B, L, 1, dtype=torch.bool, device=dev)
    reset[:, 0] = True
    with torch.no_grad():
        ms_obs = timed(lambda: r.observe(embed, action, r.initial(B), reset, seed=5))
    b_obs = 4.0 * L * (numel(r._deter_net) + numel(r._obs_net))
    f_upd = UPDATE_FLOP.get((cfg_name, B, L, H))
    out = {
        "imagination": {"bound": "mfma", "latents_per_s": N * H / (ms_img * 1e-3), "ms": ms_img,
                        "achieved": f_img / (ms_img * 1e-3) / 1e12, "peak": 157.3, "unit": "TFLOP/s",
                        "frac": f_img / (ms_img * 1e-3) / 1e12 / 157.3, "work": f_img,
                        "what": f"_imagine_tm: N={N} start rows, H={H} img_steps + {H + 1} actor samples, alone"},
        # the weights stream from L2/MALL, so the HBM fraction is no bound; the real bound is the dependent launch
        # chain: 5 fused launches per step, each >= one kernel boundary (1.45 us between trivial kernels,
        # MI355X_MICROARCH.md price list row 'boundary') plus its dependent prologue load (~1 us, an L2 round trip)
        "observe_scan": {"bound": "launch latency", "ms": ms_obs, "launches": 5 * L,
                         "latency_floor_ms": 5 * L * (1.45 + 1.0) * 1e-3,
                         "frac": 5 * L * (1.45 + 1.0) * 1e-3 / ms_obs,
                         "weight_stream_GBps": b_obs / (ms_obs * 1e-3) / 1e9, "work": b_obs,
                         "what": f"RSSM.observe forward, B={B} L={L}: 5 dependent launches per step; weight bytes "
                                 "(Deter + obs_net once per step) over the phase time as weight_stream_GBps"},
    }
    if f_upd:  # only where the update's FLOP were counted on the reference
        out["update"] = {"bound": "mfma", "achieved": f_upd / (ms_update * 1e-3) / 1e12, "peak": 157.3,
                         "unit": "TFLOP/s", "frac": f_upd / (ms_update * 1e-3) / 1e12 / 157.3, "work": f_upd,
                         "what": f"whole Dreamer.update, {f_upd / 1e9:.1f} GFLOP fwd+bwd (SURVEY §8(d)) / ms_per_step"}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="dmc/cnn", choices=sorted(WORKLOADS))
    ap.add_argument("--global-batch", action="store_true",
                    help="divide the config's batch_size over the ranks (strong scaling of the batch) instead of "
                         "keeping it per GPU (weak scaling, the default)")
    ap.add_argument("--cpu-updates", type=int, default=3)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--backend", default="nccl", help="nccl (= RCCL); gloo only to rehearse N ranks on one GPU")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    local = local % max(torch.cuda.device_count(), 1)  # == LOCAL_RANK on a node with one GPU per rank
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group(args.backend)

    from sdreamer import kernels as K
    from sdreamer.config import load_config
    from sdreamer.dreamer import Dreamer

    A, discrete, workload = WORKLOADS[args.config]
    ovr = [f"device=cuda:{local}", "model.compile=False"]
    B0 = int(load_config(args.config, ovr).batch_size)
    if args.global_batch:
        if B0 % world:
            raise SystemExit(f"--global-batch: batch_size {B0} does not split over {world} ranks")
        ovr.append(f"batch_size={B0 // world}")
    cfg = load_config(args.config, ovr)
    B, L, H = int(cfg.batch_size), int(cfg.batch_length), int(cfg.model.imag_horizon)
    torch.manual_seed(0)  # identical initial weights on every rank
    act_space = _Sp((A,))
    if discrete:
        act_space.discrete = True
    agent = Dreamer(cfg.model, _Spaces({"image": _Sp((64, 64, 3))}), act_space, rank=rank, world=world)
    buf = synth_buffer(cfg, device, rank, T=max(160, 2 * (L + 1)), A=A, discrete=discrete)

    # roofline probe on the dominant kernel: sees its launch (eager warm-up or graph capture), then re-times that
    # exact launch with HIP events on its stream after the timed steps
    probe = None if args.no_roofline else dominant_probe(K)
    for _ in range(args.warmup):
        agent.update(buf)
    trace_mark(1)  # kernel-trace window of the timed steps (tools/kernel_table.py); outside the timed region
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
    trace_mark(2)
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
        "ms_per_step": ms, "higher_is_better": True, "scaling": "strong" if args.global_batch else "weak",
        "vs_baseline": None, "dtype": "f32 (split-bf16 gradient GEMMs)",
        "precision": "fp32 everywhere a sampled index or a WM loss depends on (fp32 MFMA, and the fp32-accurate "
                     "3-way split-bf16 'bf16x6' MFMA in the imagination); gradient contractions and the frozen "
                     "imagined heads on 2-way split-bf16 (~1e-5 rel); DESIGN.md §2",
        "data": "synthetic (uniform uint8 64x64x3 images, " + ("one-hot uniform" if discrete else "U(-1,1)") +
                " actions, U(0,1) rewards; random-init weights)",
        "config": {"workload": f"{workload}, per-GPU B{B} L{L} H{H}", "config": args.config,
                   "global_batch": B * world, "per_gpu_batch": B, "seq_len": L, "imag_horizon": H,
                   "parallelism": f"dp{world}"},
    }
    if probe is not None:
        # the dominant kernel (k_lin, imagination) and, as secondary entries, the other two imagination contractions
        # and the largest single MFMA launch (encoder stage 2); HBM bytes per launch from separate rocprofv3 --pmc
        # FETCH_SIZE / WRITE_SIZE passes (tools/roofline_traffic.py: gfx950 FETCH_SIZE x2), committed under profiles/
        import glob
        out["roofline"] = imag_kernel_probe(agent, cfg, 0)
        out["roofline_secondary"] = {"k_hid": imag_kernel_probe(agent, cfg, 1),
                                     "k_gate": imag_kernel_probe(agent, cfg, 2), "conv_stage2": probe.report()}
        tfs = sorted(glob.glob(os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles",
                                            "r*_roofline_traffic.json")))
        tf = tfs[-1] if tfs else ""
        if tf:
            tj = json.load(open(tf))
            for ent in [out["roofline"]] + list(out["roofline_secondary"].values()):
                t = tj.get(ent.get("key", "conv_fwd_direct_pool")) if ent else None
                if t and t.get("traffic_bytes"):
                    ent["traffic"] = t["traffic_bytes"]
                    ent["traffic_source"] = f"profiles/{os.path.basename(tf)} (rocprofv3 --pmc)"
                    ent["algorithmic_bytes"] = t.get("algorithmic_bytes")
            out["roofline"].setdefault("traffic", None)
    if not args.no_roofline:
        out["phases"] = phase_rooflines(agent, cfg, args.config, ms)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        if args.config == "dmc/cnn":  # checker legs beside the CPU baseline
            out["parity"] = wm_loss_parity_full()
            out["parity_golden_small"] = wm_loss_parity()
        # every core of this process's affinity, capped by the box's CPU share (OMP_NUM_THREADS, 16 per GPU there)
        share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
        aff = len(os.sched_getaffinity(0))
        threads = min(aff, share) if share > 0 else aff
        cfg_cpu = load_config(args.config, ["device=cpu", "model.compile=False", f"batch_size={B}"])
        t_cpu = cpu_baseline(cfg_cpu, args.cpu_updates, threads, A, discrete)
        out["cpu_baseline"] = {"value": B * L * H / t_cpu, "unit": "imagined_latents/s", "cores": threads,
                               "kind": "port", "cpu": cpu_model(), "affinity_cores": aff,
                               "sample": f"oracle/ref_cpu.py OracleAgent.update() at walker B{B} L{L} H{H} fp32, "
                                         f"median of {args.cpu_updates} after 1 warm-up ({t_cpu:.2f} s/update)"}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
