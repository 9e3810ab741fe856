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
SCAN_SKELETON_US = 15.8  # 4 graph-captured launches per observe step, <= 32 KB weights + 32 KB operands each (r04 prototype)
# split-bf16 ("bf16x3") kernels: three v_mfma_f32_16x16x32_bf16 per f32-equivalent product, so their f32-equivalent
# peak is the dense bf16 MFMA peak (2.5 PFLOP/s, MI355X_MICROARCH.md) / 3
PEAK_BF16X3 = 2500.0 / 3
PEAK_BF16X6 = 2500.0 / 6  # the imagination's k_hid / k_gate / k_lin6: six bf16 MFMAs per f32-equivalent product


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


# the parity legs run a fresh agent's FIRST update, which is eager (graphs are captured after two eager updates); the
# timed updates replay the graphs. tests/test_gpu_graph_fullsize.py pins graph replay == eager bit for bit (metrics,
# parameters, replay storage over 5 updates at C2 / C4 / C5), which is what carries these numbers to the timed path.
EAGER_NOTE = "eager first update; graph replay == eager bit-exact (tests/test_gpu_graph_fullsize.py, C2/C4/C5)"


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
                                    f"B{int(z['meta_B'])} L{int(z['meta_T'])} H{int(z['meta_H'])})",
            "path": EAGER_NOTE}


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
                    f"B{B} L{L} H{H}, same weights / batch / noise seed)", "path": EAGER_NOTE}


# The committed kernel table of this build (tools/profile_round.sh -> tools/kernel_table.py: the rocprofv3 kernel trace
# of a bench run, windowed to its timed steps, joined with the separate --pmc passes). Named explicitly, never "the
# newest file": its rows rank the update's launch shapes by time per update and carry their counter traffic.
KERNEL_TABLE = "profiles/r06final/r06final_kernel_table.json"


def clock_probe(nwg=256, iters=20000, reps=3):
    """Shader clock under an f32-MFMA load (sd_clock_probe: per workgroup s_memtime cycles / s_memrealtime ticks around
    an MFMA loop, MI355X_MICROARCH.md 'DVFS give-back' item 6): median over workgroups of the last of `reps` launches."""
    from sdreamer import _native as nat
    from sdreamer import kernels as K
    stamps = torch.zeros(2 * nwg, dtype=torch.int64, device="cuda")
    sink = torch.empty(nwg, device="cuda")
    for _ in range(reps):
        nat.call("sd_clock_probe", stamps.data_ptr(), sink.data_ptr(), nwg, iters, K.stream())
    torch.cuda.synchronize()
    st = stamps.view(nwg, 2).cpu().double()
    ghz = (st[:, 0] / st[:, 1].clamp_min(1) * 0.1).median().item()
    return round(ghz, 3)


class _ImagStep:
    """sd_imagine_step_kernel: one launch of an imagination step's kernel (0 k_lin, 1 k_hid, 2 k_gate) re-issued after a
    run at the update's shape (same descriptor, workspace and grid), back to back between two HIP events on the stream
    it is launched on (per-launch event pairs would add the events' own cost to every launch)."""

    def __init__(self, agent, cfg):
        r = agent.rssm
        B, L, H = int(cfg.batch_size), int(cfg.batch_length), int(cfg.model.imag_horizon)
        self.N, self.H1, dev = B * L, H + 1, agent.device
        g = torch.Generator(device=dev).manual_seed(11)
        idx = torch.randint(0, r._discrete, (self.N, r._stoch), device=dev, generator=g)
        SK, D = r.flat_stoch, r._deter
        feats = torch.empty(self.H1, self.N, SK + D, device=dev)
        actions = torch.empty(self.H1, self.N, agent.act_dim, device=dev)
        feats[0, :, :SK] = torch.nn.functional.one_hot(idx, r._discrete).float().reshape(self.N, SK)
        feats[0, :, SK:] = torch.randn(self.N, D, device=dev, generator=g)
        self.keep = {}
        with torch.no_grad():
            agent._imagine_fused(feats, actions, self.H1, 5, 0, keep=self.keep)
        torch.cuda.synchronize()

    def time(self, which, reps=30):
        import ctypes
        from sdreamer import _native as nat
        from sdreamer import kernels as K
        desc = self.keep["desc"]
        H = self.H1 - 1
        # k_gate rewrites feats(t + 1): only t = H - 1 reproduces the run's values (the probe times, it keeps no output)
        ts = [H - 1] * reps if which == 2 else [i % H for i in range(reps)]
        nat.call("sd_imagine_step_kernel", ctypes.addressof(desc), which, ts[0], K.stream())  # warm
        return _graph_us(lambda i: nat.call("sd_imagine_step_kernel", ctypes.addressof(desc), which, ts[i],
                                            K.stream()), reps)


def _graph_us(fn, reps):
    """Per-call device time of `fn(i)` (one kernel launch on the current stream) issued `reps` times back to back from
    one captured HIP graph, median of 5 replays timed with HIP events on the graph's stream: the kernel plus the
    stream's launch boundary, with no host launch overhead between the calls (a ctypes call per launch costs more host
    time than these step kernels take)."""
    g = torch.cuda.CUDAGraph()
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    with torch.cuda.graph(g, stream=st):
        for i in range(reps):
            fn(i)
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    ts = []
    with torch.cuda.stream(st):
        for _ in range(5):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record(st)
            g.replay()
            e.record(st)
            torch.cuda.synchronize()
            ts.append(s.elapsed_time(e) / reps * 1e3)
    return sorted(ts)[2]


class _ScanStep:
    """sd_rssm_scan_step_kernel: one launch of an observe-scan forward phase (0 x1p slab, 1 k_hid, 2 k_gate, 3 obs_net_0 +
    next x0p slab, 4 k_logit) at step T - 1, re-issued after an eager RSSM.observe at the update's shape."""

    def __init__(self, agent, cfg):
        from sdreamer import rssm as R
        r = agent.rssm
        B, L = int(cfg.batch_size), int(cfg.batch_length)
        dev = agent.device
        g = torch.Generator(device=dev).manual_seed(13)
        embed = torch.randn(B, L, r.embed_size, device=dev, generator=g)
        action = torch.rand(B, L, r._act_dim, device=dev, generator=g) * 2 - 1
        reset = torch.zeros(B, L, 1, dtype=torch.bool, device=dev)
        reset[:, 0] = True
        R.SCAN_KEEP = {}
        try:
            with torch.no_grad():
                self.out = r.observe(embed, action, r.initial(B), reset, seed=5)
            torch.cuda.synchronize()
            self.keep = R.SCAN_KEEP
        finally:
            R.SCAN_KEEP = None
        self.ok = "desc" in self.keep

    def time(self, which, reps=40):
        import ctypes
        from sdreamer import _native as nat
        from sdreamer import kernels as K
        desc = self.keep["desc"]
        t = self.keep["T"] - 1
        nat.call("sd_rssm_scan_step_kernel", ctypes.addressof(desc), which, t, K.stream())
        return _graph_us(lambda i: nat.call("sd_rssm_scan_step_kernel", ctypes.addressof(desc), which, t, K.stream()),
                         reps)


def probe_specs(agent, cfg, K):
    """The update's largest launch shapes that bench.py can re-time live, keyed by the kernel-table row they match
    (demangled name, launch grid in workgroups). Each entry: bound, work per launch (FLOP or bytes), algorithmic bytes
    per launch (every operand read once, every output written once), and how to time it. LaunchProbes must exist
    before the warm-up updates (they record the launch while the update's graphs are captured)."""
    r = agent.rssm
    B, L, H = int(cfg.batch_size), int(cfg.batch_length), int(cfg.model.imag_horizon)
    N, D, U, SK, G, A = B * L, r._deter, r._hidden, r.flat_stoch, r._blocks, agent.act_dim
    Dg, Ig, F = D // G, D // G + 3 * U, SK + D
    ksd, kss = 8, 8  # split-K slabs of x0p (k_slab, rssm.SCAN_KSD) and x1p (k_logit_rows' categorical groups, SD_LR_NG)
    out = []

    def add(key, name, grid, bound, work, algo, label, how, launches, peak=None, alt_peak=None):
        out.append(dict(key=key, name=name, grid=list(grid), bound=bound, work=work, algo=algo, label=label, how=how,
                        launches=launches, peak=peak, alt_peak=alt_peak))

    # encoder stage 2 forward (conv + pool + RMSNorm + SiLU, direct conv from an LDS patch; on bf16x6 by default)
    cp = dominant_probe(K)
    if K.ops_fused_pool():
        pix = N * 32 * 32
        c6 = bool(K.CONV6)
        tiles = N * 32 * 32 // 512  # the ring kernel's 512-pixel tiles (64 pixels per wave), one per workgroup
        add("conv_stage2", "conv_fwd6r_direct_pool<48, 32, 5, 5, true, false, 1, 4, 32, 512>" if c6 else
            "conv_fwd_direct_pool<48, 32, 5, 5, 1>", ((tiles + 7) // 8 * 8 if c6 else N * 32 * 32 // 128, 1, 1), "mfma", 2.0 * pix * 48 * 25 * 32, 4.0 * pix * 32 + N * 16 * 16 * (48 * 9 + 4),
            cp.label, ("launch", cp), 1, peak=PEAK_BF16X6 if c6 else None, alt_peak=PEAK_FP32_MFMA if c6 else None)
    # encoder stage 2 bwd-data (split-bf16 direct conv from a pre-split dOut patch in LDS): sd_conv2d_dgrad_direct(dout,
    # wsplit, din, Nb, Hs, Ws, Ci = dout channels, Co = din channels, kh, kw, pad, stream)
    dg = K.LaunchProbe("sd_conv2d_dgrad_direct", lambda a: a[6] == 48 and a[7] == 32,
                       lambda a: 2.0 * a[3] * a[4] * a[5] * a[6] * a[7] * a[8] * a[9],
                       label="conv_dgrad3_direct<48, 2, 5, 5, 4, true, 512> (encoder stage 2 bwd-data: dOut 48 ch -> "
                             "dIn 32 ch at 32x32, 5x5 flipped weight; direct conv over 512-pixel tiles of 64-pixel "
                             "waves, the dOut patch of 16 rows split once into (hi, lo) bf16 planes in LDS, the "
                             "pre-split weight through an LDS ring, 3 v_mfma_f32_16x16x32_bf16 per f32-equivalent "
                             "product)")
    pix = N * 32 * 32
    add("conv_stage2_dgrad", "conv_dgrad3_direct<48, 2, 5, 5, 4, true, 512>", (pix // 512, 1, 1), "mfma",
        2.0 * pix * 48 * 25 * 32,
        4.0 * (pix * 48 + pix * 32) + 2.0 * 2 * 32 * 1216, dg.label, ("launch", dg), 1, peak=PEAK_BF16X3)
    # imagined heads' first layers: one split-bf16 MLP-layer launch, A = the imagined feats broadcast over 4 weights
    M = N * (H + 1)
    hp = K.LaunchProbe("sd_gemm_bf16x3_mlp", lambda a: a[0]._obj.batch == 4 and a[0]._obj.strideA == 0,
                       lambda a: 2.0 * a[0]._obj.M * a[0]._obj.N * a[0]._obj.K * a[0]._obj.batch,
                       label="gemm3_w256_kernel (imagined reward / continue / value / slow-value first layers: "
                             "(M, F) x 4 (F, U) split-bf16, 256 x 256 tiles on v_mfma_f32_32x32x16_bf16, per-entry "
                             "weights, row partials for the next layer's RMSNorm; 3 bf16 MFMAs per f32-equivalent "
                             "product)")
    # (the 256 x 256-tile kernel where one 256-wide entry per tile fills the chip: gemm3.hip SD_MLP_W256)
    w256 = U == 256 and -(-M // 256) * 4 >= 192
    add("heads_l0", "gemm3_w256_kernel<true>" if w256 else "gemm3_mlp_kernel<false, true, 128>",
        (-(-M // 256) * 4, 1, 1) if w256 else (U // 128, M // 128, 4), "mfma",
        2.0 * M * F * U * 4, 4.0 * (M * F + 4 * F * U + 4 * M * U + 4 * (U // 64) * M), hp.label, ("launch", hp), 1,
        peak=PEAK_BF16X3)
    # imagination step kernels
    # k_lin6 (pre-split deter image + weight images, 32-row tiles) unless SDHIP_KL_NOPRE selects the fp32 k_lin
    # (k_lin6_areg — 64 x 48 tiles over the three problems' columns, K split over two halves of a 512-thread
    # workgroup — at D = 2048 / 4096, U = 256)
    lin6 = not os.environ.get("SDHIP_KL_NOPRE")
    lareg = lin6 and D in (2048, 4096) and U == 256 and not os.environ.get("SDHIP_KL_NOAREG")
    imag = [("imag_k_lin", "k_lin6_areg" if lareg else "k_lin6<32, 32>" if lin6 else "k_lin<32, 32>",
             (3 * U // 48, N // 64, 1) if lareg else (U // 32, N // 32, 3),
             3 * 2.0 * N * D * U, 4.0 * (N * D + 3 * U * D + 3 * N * U + 2 * (U // 16) * N),
             IMAG_LABELS[4 if lareg else 3 if lin6 else 0], 0),
            ("imag_k_hid", "k_hid_areg" if (Ig // 32 in (32, 40) and not os.environ.get("SDHIP_KH_NOAREG"))
             else "k_hid", (D // 64, N // 64, 1), 2.0 * N * D * Ig,
             4.0 * (N * D + 3 * N * U + D * Ig + N * D + N * D // 64), IMAG_LABELS[1], 1),
            ("imag_k_gate", "k_gate", (D // 32, N // 64, 1), 2.0 * N * 3 * D * Dg,
             4.0 * (N * D + 3 * D * Dg + 2 * N * D), IMAG_LABELS[2], 2)]
    for key, name, grid, work, algo, label, which in imag:  # the bf16x6 ceiling they run on (alt: the f32 peak)
        x6 = not (which == 0 and not lin6)
        add(key, name, grid, "mfma", work, algo, label, ("imag", which), H,
            peak=PEAK_BF16X6 if x6 else None, alt_peak=PEAK_FP32_MFMA if x6 else None)
    # observe-scan forward phases (M = B rows: weight-streaming, bytes-bound)
    scan = [("scan_k_hid", "k_hid<8, 2, true, 16>", (D // 16, 1, 1), 4.0 * (D * Ig + 2 * B * D + (2 + kss + 1) * B * U),
             "scan k_hid (RSSM.observe step: _dyn_hid BlockLinear, M = B rows, 16-column tiles; x0 / x1 RMSNorm + SiLU "
             "prologue)", 1),
            ("scan_k_gate", "k_gate<2, 2, 8, 16>", (D // 8, 1, 1), 4.0 * (3 * D * Dg + 8 * B * D),
             "scan k_gate (_dyn_gru BlockLinear + GRU epilogue, M = B rows, 8 deter columns x 3 gates per workgroup)", 2),
            ("scan_k_logit", "k_logit_rows<%d, %d>" % (r._discrete, SK // (kss * r._discrete)), (kss, B, 1),
             4.0 * (2 * SK * U + (ksd + 1) * B * U + 5 * B * SK + 6 * B * U),
             "scan k_logit_rows (RSSM.observe step: obs_net RMSNorm + logits + unimix one-hot sampler by (categorical "
             "group, row), and the next step's _dyn_in1 as a gather of the sampled W1^T rows, staged in LDS)", 4),
            ("scan_k_slab_obs", "k_slab<2>", (U // 16, ksd, 2), 4.0 * (2 * U * D + B * D + 2 * ksd * B * U),
             "scan k_slab (obs_net_0 deter half + next _dyn_in0, split-K slabs)", 3)]
    for key, name, grid, algo, label, which in scan:
        add(key, name, grid, "hbm", algo, algo, label, ("scan", which), L)
    return out


IMAG_LABELS = {
    0: "k_lin<32, 32> x3 (imagination step: img_net_0 + _dyn_in0 + actor layer 0's deter part, three (N, D) x (D, U) "
       "GEMMs in one launch, RMSNorm row partials in the epilogue; v_mfma_f32_16x16x4_f32)",
    1: "k_hid_areg (imagination step: _dyn_hid BlockLinear, K = Dg + 3U per block; A fragments loaded per lane from the "
       "pre-split deter / x0 / x1 / x2 images, the weight tile through LDS; bf16x6)",
    2: "k_gate (imagination step: _dyn_gru BlockLinear + GRU epilogue, RMSNorm + SiLU of hp in the A loader; bf16x6)",
    3: "k_lin6<32, 32> x3 (imagination step: img_net_0 + _dyn_in0 + actor layer 0's deter part, three (N, D) x (D, U) "
       "GEMMs in one launch on pre-split bf16x6 operands — the deter image k_gate writes, weight images split once per "
       "imagination — RMSNorm row partials in the epilogue; 6 v_mfma_f32_16x16x32_bf16 per f32-equivalent product)",
    4: "k_lin6_areg x3 (imagination step: img_net_0 + _dyn_in0 + actor layer 0's deter part, three (N, D) x (D, U) "
       "GEMMs in one launch, 64 x 48 tiles over their concatenated columns (256 workgroups of 512 threads, the K range "
       "split over two halves); deter fragments "
       "loaded per lane from the pre-split image, weight tiles through LDS; bf16x6)",
}


class FlopCensus:
    """Counts the algorithmic FLOP of one eager update by the arithmetic that executes them, from the C-ABI calls
    (registered in _native.PROBES): split-bf16 ("bf16x3") GEMMs / MLP layers / weight gradients / conv bwd-data and
    bwd-weight, the imagination's three bf16x6 step contractions (k_hid, k_gate, k_lin6 per step), and everything
    else exact f32. Gives phases.update its precision-weighted ceiling: the time the update's FLOP would take at the
    peak of the arithmetic each part runs on."""

    X3 = ("sd_gemm_bf16x3_wgrad", "sd_gemm_bf16x3_wgrad2", "sd_gemm_bf16x3_mlp", "sd_conv2d_dgrad_bf16x3",
          "sd_conv2d_dgrad_direct", "sd_conv2d_wgrad_bf16x3")

    def __init__(self, agent):
        r = agent.rssm
        self.D, self.U, self.G = r._deter, r._hidden, r._blocks
        self.flop = {"f32": 0.0, "bf16x3": 0.0, "bf16x6": 0.0}

    def match(self, name, args):
        if name.startswith(("sd_gemm", "sd_conv2d", "sd_imagine_run")):
            self._name = name
            return True
        return False

    def begin(self):
        pass

    def end(self, args):  # after the launch (call_shaped skips it when the entry point declined the shape)
        self.record(self._name, args)

    def record(self, name, args):
        if name in ("sd_gemm_f32", "sd_gemm_bf16x3") or name in self.X3[:3]:
            d = args[0]._obj if hasattr(args[0], "_obj") else None
            if d is None:
                return
            f = 2.0 * d.M * d.N * d.K * d.batch
            x3 = name != "sd_gemm_f32" and (name != "sd_gemm_bf16x3" or min(d.M, d.N, d.K) >= 64)
            self.flop["bf16x3" if x3 else "f32"] += f
        elif name in ("sd_conv2d_fwd_pool", "sd_conv2d_fwd_pool6"):  # (in, w, b, nw, pooled, amax, y, rstd, Nb, ...)
            Nb, Hs, Ws, Ci, Co, kh, kw = args[8:15]
            self.flop["bf16x6" if name.endswith("6") else "f32"] += 2.0 * Nb * Hs * Ws * Co * kh * kw * Ci
        elif name == "sd_conv2d_fwd":  # (in, w, b, out, Nb, Hs, Ws, Ci, Co, kh, kw, pad, ups)
            Nb, Hs, Ws, Ci, Co, kh, kw, _, ups = args[4:13]
            self.flop["f32"] += 2.0 * Nb * (Hs << ups) * (Ws << ups) * Co * kh * kw * Ci
        elif name in ("sd_conv2d_dgrad_bf16x3", "sd_conv2d_dgrad_direct"):  # (dout, w, din, Nb, Hs, Ws, Ci, Co, kh, kw)
            Nb, Hs, Ws, Ci, Co, kh, kw = args[3:10]
            self.flop["bf16x3"] += 2.0 * Nb * Hs * Ws * Ci * Co * kh * kw
        elif name == "sd_conv2d_wgrad_bf16x3":  # (in, dout, dw_db, ws, wsf, Nb, Hs, Ws, Ci, Co, kh, kw, ...)
            Nb, Hs, Ws, Ci, Co, kh, kw = args[5:12]
            self.flop["bf16x3"] += 2.0 * Nb * Hs * Ws * Ci * Co * kh * kw
        elif name == "sd_conv2d_wgrad":  # (in, dout, dw_db, ws, wsf, ksplit, Nb, Hs, Ws, Ci, Co, kh, kw, pad, ups)
            Nb, Hs, Ws, Ci, Co, kh, kw, _, ups = args[6:15]
            self.flop["f32"] += 2.0 * Nb * (Hs << ups) * (Ws << ups) * Ci * Co * kh * kw
        elif name == "sd_conv2d_wgrad_pool":  # (in, dpool, amax, dw_db, ws, wsf, Nb, H, W, Ci, Co, kh, kw, ...)
            Nb, H_, W_, Ci, Co, kh, kw = args[6:13]
            self.flop["f32"] += 2.0 * Nb * H_ * W_ * Ci * Co * kh * kw
        elif name == "sd_imagine_run":  # per img_step: _dyn_hid, _dyn_gru and the three (N, D) x (D, U) contractions
            import ctypes
            from sdreamer import _native as nat
            d = ctypes.cast(args[0], ctypes.POINTER(nat.ImagineDesc)).contents if isinstance(args[0], int) else \
                args[0]._obj
            D, U, G = self.D, self.U, self.G
            Dg = D // G
            per_step = D * (Dg + 3 * U) + 3 * D * Dg + 3 * D * U
            self.flop["bf16x6"] += 2.0 * d.N * (d.H1 - 1) * per_step

    def ceiling(self, total):
        """(ms at the precision-weighted peak, FLOP per class): the f32 class is the reference's counted total minus
        the split-bf16 classes (the scan, encoder forward, WM-loss contractions, samplers and the imagination's small
        kernels run exact f32)."""
        x3, x6 = self.flop["bf16x3"], self.flop["bf16x6"]
        f32 = max(total - x3 - x6, 0.0)
        ms = (f32 / (PEAK_FP32_MFMA * 1e12) + x3 / (PEAK_BF16X3 * 1e12) + x6 / (PEAK_BF16X6 * 1e12)) * 1e3
        return ms, {"f32": f32, "bf16x3": x3, "bf16x6": x6, "census_f32": self.flop["f32"]}


def _kernel_is(row_name, name):
    """A kernel-table row's name (demangled, or the mangled symbol of a kernel in an anonymous namespace) is `name`
    (the table's spelling: 'k_lin6<32, 32>', or a bare 'k_hid' for a mangled row)."""
    if row_name.startswith(name):
        return True
    base = name.split("<")[0]
    return row_name.startswith("_Z") and (f"{len(base)}{base}I" in row_name or f"{len(base)}{base}E" in row_name)


def roofline_entries(specs, agent, cfg, table):
    """Time every probe spec live and join it with its kernel-table row. Returns the entries ordered by the table's
    per-update rank (live per-update time when there is no table)."""
    imag = scan = None
    rows = table["rows"] if table else []
    res = []
    for sp in specs:
        kind = sp["how"][0]
        if kind == "launch":
            pr = sp["how"][1]
            pr.stop()
            pr.replay(20)
            rep = pr.report()
            if rep is None:
                continue
            avg_us = rep["avg_us"]
        elif kind == "imag":
            imag = imag or _ImagStep(agent, cfg)
            avg_us = imag.time(sp["how"][1])
        else:
            scan = scan or _ScanStep(agent, cfg)
            if not scan.ok:
                continue
            avg_us = scan.time(sp["how"][1])
        peak = sp["peak"] or (PEAK_FP32_MFMA if sp["bound"] == "mfma" else PEAK_HBM)
        unit = "TFLOP/s" if sp["bound"] == "mfma" else "GB/s"
        achieved = sp["work"] / (avg_us * 1e-6) / (1e12 if unit == "TFLOP/s" else 1e9)
        e = {"key": sp["key"], "kernel": sp["label"], "symbol": sp["name"], "grid": sp["grid"], "bound": sp["bound"],
             "achieved": achieved, "peak": peak, "unit": unit, "frac": achieved / peak, "avg_us": avg_us,
             "work_per_launch": sp["work"], "algorithmic_bytes": sp["algo"], "traffic": None,
             "timing": ("the update's own launch re-issued 20x from its captured graph node, HIP events"
                        if kind == "launch" else "40 / 30 back-to-back launches from one captured HIP graph, HIP "
                        "events: kernel + the stream's launch boundary (the trace's avg us is the kernel alone)")}
        if sp.get("alt_peak"):  # `peak` is the ceiling of the arithmetic the kernel executes (bf16x6: 6 bf16 MFMAs
            # per f32-equivalent product); alt = the same FLOP against the f32 MFMA peak
            e.update(alt_peak=sp["alt_peak"], frac_alt=achieved / sp["alt_peak"], alt_is="f32 MFMA peak")
        e["arith"] = ("bf16x6" if peak == PEAK_BF16X6 else "bf16x3" if peak == PEAK_BF16X3 else
                      "f32" if sp["bound"] == "mfma" else "bytes")
        row = next(((i, rw) for i, rw in enumerate(rows)
                    if _kernel_is(rw["kernel"], sp["name"]) and rw["grid"] == sp["grid"]), None)
        if row:
            i, rw = row
            e.update(rank=i + 1, launches_per_update=rw["launches_per_update"],
                     trace_avg_us=rw["avg_us"], trace_ms_per_update=rw["ms_per_update"],
                     frac_trace=sp["work"] / (rw["avg_us"] * 1e-6) / (1e12 if unit == "TFLOP/s" else 1e9) / peak,
                     traffic=rw.get("hbm_bytes"), mfma_util=rw.get("mfma_util"),
                     trace_clock_ghz=rw.get("clock_ghz") if (rw.get("clock_ghz") or 9.0) <= 2.4 else None,
                     trace_clock_source=rw.get("clock_source"),
                     l2_hit=rw.get("l2_hit"), traffic_source=f"{KERNEL_TABLE} (rocprofv3 --pmc FETCH_SIZE x2 + "
                                                             "WRITE_SIZE, per dispatch)")
            if e["traffic"]:
                e["traffic_over_algorithmic"] = e["traffic"] / sp["algo"]
            if sp.get("alt_peak"):
                e["frac_alt_trace"] = e["frac_trace"] * peak / sp["alt_peak"]
        else:
            e["launches_per_update"] = sp["launches"]
        e["ms_per_update"] = e["avg_us"] * e["launches_per_update"] / 1e3
        res.append(e)
    if rows:
        res.sort(key=lambda e: e.get("rank", 10 ** 6))
    else:
        res.sort(key=lambda e: -e["ms_per_update"])
    return res


def dominant_probe(K):
    """Roofline probe of the encoder's second stage forward, conv + MaxPool2d(2) + RMSNorm2D + SiLU in one launch
    (direct conv, M = B*L*32*32 pixels, N = 48, K = 5*5*32), the update's largest single MFMA launch.
    Algorithmic work = 2*M*N*K FLOP per launch."""
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
    if K.CONV6:  # sd_conv2d_fwd_pool6: the same arguments with the split weight image in place of w
        return K.LaunchProbe("sd_conv2d_fwd_pool6", lambda a: a[11] == 32 and a[12] == 48, flops,
                             label="conv_fwd6r_direct_pool<48, 32, 5, 5> (encoder stage 2: 32->48 ch, 32x32, 5x5 "
                                   "conv + 2x2 max-pool + RMSNorm + SiLU epilogue; direct conv over 512-pixel tiles "
                                   "from the input patch staged once as three bf16 planes, the pre-split weight "
                                   "through an LDS ring shared by 8 waves; bf16x6 = 6 v_mfma_f32_16x16x32_bf16 per "
                                   "f32-equivalent product, fp32-accurate)")
    return K.LaunchProbe("sd_conv2d_fwd_pool", lambda a: a[11] == 32 and a[12] == 48, flops,
                         label="conv_fwd_direct_pool<48> (encoder stage 2: 32->48 ch, 32x32, 5x5 conv + 2x2 max-pool + "
                               "RMSNorm + SiLU epilogue; direct conv from an LDS input patch, v_mfma_f32_16x16x4_f32, "
                               "N tile = 48)")


def phase_rooflines(agent, cfg, cfg_name, ms_update, table=None, reps=10, census=None):
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
        # the observe scan against the HBM roofline (the north star's 'achieved HBM GB/s on the recurrent scan'):
        # algorithmic bytes = the Deter + obs_net weights streamed once per step; what actually bounds it is the
        # dependent launch chain (4 launches per step), so the same time is also given against the measured floor of
        # 4 graph-captured launches per step that each stage <= 32 KB of weights and <= 32 KB of activations
        # (15.8 us per step, tools/hip/persist_scan_proto.hip, profiles/r04_persist_proto.txt)
        "observe_scan": {"bound": "launch latency", "ms": ms_obs, "launches": 4 * L, "work": b_obs,
                         "us_per_step": ms_obs * 1e3 / L,
                         "skeleton_floor_ms": L * SCAN_SKELETON_US * 1e-3,
                         "frac_of_skeleton_floor": L * SCAN_SKELETON_US * 1e-3 / ms_obs,
                         # NOT a bound: the weights stream from L2 / MALL and the dependent chain of 4 launches per
                         # step is what sets the time; the algorithmic weight bytes over the phase time, against HBM
                         "algorithmic_GBps": b_obs / (ms_obs * 1e-3) / 1e9,
                         "algorithmic_frac_of_hbm": b_obs / (ms_obs * 1e-3) / 1e9 / PEAK_HBM, "hbm_peak": PEAK_HBM,
                         "what": f"RSSM.observe forward, B={B} L={L}: 4 dependent launches per step; algorithmic bytes "
                                 "= Deter + obs_net weights once per step"},
    }
    if table:  # counter bytes of the scan forward's kernels (k_slab / k_hid / k_gate / k_logit of the fused scan) from the
        # committed PMC passes, per update, over the live phase time: the 'achieved HBM GB/s on the recurrent scan'
        scan_rows = [rw for rw in table["rows"]
                     if rw["kernel"].split("<")[0] in ("k_slab", "k_logit", "k_logit_rows", "k_init", "k_hid", "k_gate")]
        cb = sum(rw.get("hbm_bytes", 0.0) * rw["launches_per_update"] for rw in scan_rows)
        tm = sum(rw["ms_per_update"] for rw in scan_rows)
        hit = [(rw.get("l2_hit"), rw["ms_per_update"]) for rw in scan_rows if rw.get("l2_hit") is not None]
        out["observe_scan"].update(
            counter_bytes_per_update=cb, counter_GBps=cb / (ms_obs * 1e-3) / 1e9,
            counter_frac_of_hbm=cb / (ms_obs * 1e-3) / 1e9 / PEAK_HBM,
            trace_kernel_ms_per_update=tm,
            l2_hit_time_weighted=(sum(h * t for h, t in hit) / sum(t for _, t in hit)) if hit else None,
            counter_source=f"{KERNEL_TABLE}: scan forward kernels' HBM bytes per dispatch x dispatches per update")
        heads = [rw for rw in table["rows"] if rw["kernel"].startswith("gemm3_kernel")]
        if heads:  # MFMA utilisation of the split-bf16 GEMMs (heads + gradient contractions), time-weighted
            t = sum(rw["ms_per_update"] for rw in heads)
            out["gemm3_mfma_util"] = {"time_weighted": sum(rw.get("mfma_util", 0.0) * rw["ms_per_update"]
                                                           for rw in heads) / t, "ms_per_update": t,
                                      "source": KERNEL_TABLE}
    if f_upd:  # only where the update's FLOP were counted on the reference
        out["update"] = {"bound": "mfma", "achieved": f_upd / (ms_update * 1e-3) / 1e12, "peak": 157.3,
                         "unit": "TFLOP/s", "frac": f_upd / (ms_update * 1e-3) / 1e12 / 157.3, "work": f_upd,
                         "what": f"whole Dreamer.update, {f_upd / 1e9:.1f} GFLOP fwd+bwd (SURVEY §8(d)) / ms_per_step"}
        if census is not None and sum(census.flop.values()) > 0:
            ms_c, cls = census.ceiling(f_upd)
            out["update"]["precision_weighted"] = {
                "ceiling_ms": ms_c, "frac": ms_c / ms_update, "flop": cls,
                "peaks_TFLOPs": {"f32": PEAK_FP32_MFMA, "bf16x3": PEAK_BF16X3, "bf16x6": PEAK_BF16X6},
                "what": "the update's FLOP at the peak of the arithmetic each part runs on (bench.FlopCensus over one "
                        "eager update: split-bf16 GEMMs / conv backward at 2.5 PF / 3, the imagination's bf16x6 step "
                        "contractions at 2.5 PF / 6, the rest of the reference's 927.7 GFLOP at the f32 MFMA peak) "
                        "over ms_per_step"}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="dmc/cnn", choices=sorted(WORKLOADS))
    ap.add_argument("--batch", type=int, default=0,
                    help="per-GPU batch_size override (e.g. one rank's shard of an 8-GPU global batch, timed on one GPU)")
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
    if args.batch:
        ovr.append(f"batch_size={args.batch}")
        B0 = args.batch
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

    # roofline probes on the update's largest launch shapes: LaunchProbes see their launch during the warm-up (eager
    # update or graph capture) and re-time that exact launch with HIP events on its stream after the timed steps;
    # the imagination / scan kernels are re-issued through their step entry points
    specs = None if args.no_roofline else probe_specs(agent, cfg, K)
    census = None
    if not args.no_roofline and args.warmup > 0:  # FLOP by arithmetic of the first (eager) warm-up update
        from sdreamer import _native as nat
        census = FlopCensus(agent)
        nat.PROBES.append(census)
    for i in range(args.warmup):
        agent.update(buf)
        if census is not None and i == 0:
            nat.PROBES.remove(census)
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
    table = None
    if specs is not None:
        tpath = os.path.join(ROOT, KERNEL_TABLE)
        if args.config == "dmc/cnn" and not args.global_batch and os.path.exists(tpath):
            table = json.load(open(tpath))  # profiled at this workload (tools/profile_round.sh runs bench.py defaults)
        clk0 = clock_probe()
        ents = roofline_entries(specs, agent, cfg, table)
        clk1 = clock_probe()
        # `roofline`: the update's dominant launch shape (rank 1 of the kernel table by time per update among the
        # shapes bench can re-time); `roofline_top`: the first three; every other probe in `roofline_more`
        out["roofline"] = ents[0] if ents else None
        out["roofline_top"] = ents[:3]
        out["roofline_more"] = ents[3:]
        out["kernel_table"] = {"file": KERNEL_TABLE if table else None,
                               "note": "ranks / trace_avg_us / traffic / mfma_util / clock from the committed rocprofv3 "
                                       "trace + PMC of this build at this workload; avg_us, achieved and frac are live"}
        # shader clock under an f32-MFMA load before / after the probes (sd_clock_probe, in-kernel s_memtime over
        # s_memrealtime): DVFS state of this box while the probes ran
        out["clock_ghz_mfma_load"] = [clk0, clk1]
        # per-launch time of an empty dispatch replayed the same way: the launch boundary inside the graph-timed figures
        from sdreamer import _native as nat
        out["graph_empty_dispatch_us"] = _graph_us(lambda i: nat.call("sd_trace_mark", 3, K.stream()), 40)
    if not args.no_roofline:
        out["phases"] = phase_rooflines(agent, cfg, args.config, ms, table, census=census)
        sc = out["phases"]["observe_scan"]
        # the recurrent scan beside the dominant kernel: what bounds the observe phase (the dependent launch chain),
        # its time per step against the measured 4-launch floor, and its weight bytes against HBM
        out["roofline_scan"] = {
            "bound": "launch latency", "us_per_step": sc["us_per_step"],
            "floor_us_per_step": SCAN_SKELETON_US, "frac_of_floor": sc["frac_of_skeleton_floor"],
            "algorithmic_GBps": sc["algorithmic_GBps"], "algorithmic_frac_of_hbm": sc["algorithmic_frac_of_hbm"],
            "counter_GBps": sc.get("counter_GBps"), "counter_frac_of_hbm": sc.get("counter_frac_of_hbm"),
            "what": "RSSM.observe forward alone (phases.observe_scan)"}
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
