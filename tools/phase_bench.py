"""Stand-alone timing of update phases at the bench shape (walker B16 L64 H15), HIP events on the current stream:
  * every captured phase graph of a graph-replayed update, replayed alone (its inputs persist between replays);
  * the imagined heads + lambda-returns (_heads_returns) with the fused heads path on and off, and its first-layer
    batched GEMM alone.
  * `contention`: the latency-bound critical phases beside their fillers and beside synthetic fillers.
Usage: python tools/phase_bench.py [reps] [phases, e.g. S2,M2a: only those, no heads timing | contention]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "safe-dreamer_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def contended(crit, filler, reps):
    """crit() on stream a with filler() (or nothing) on stream b started together: mean ms of crit's own span"""
    a, b = torch.cuda.Stream(), torch.cuda.Stream()
    tot = 0.0
    for i in range(reps + 1):
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(a):
            s.record()
            if filler is not None:
                b.wait_event(s)
                with torch.cuda.stream(b):
                    filler()
            crit()
            e.record()
        torch.cuda.synchronize()
        if i:
            tot += s.elapsed_time(e)
    return tot / reps


def contention(agent, reps):
    """Which property of a filler phase slows a latency-bound phase beside it: the critical S1 / M2a graphs replayed
    alone, beside their real filler (M1 / S2), beside a filler of empty dispatches (launch count only) and beside a few
    long memory-bound launches (occupancy and bandwidth only)."""
    G = dict(zip(("S0", "P", "S1", "M1", "R", "M2a", "S3", "M2b", "S4", "M2c", "M2d", "S2", "M3"), agent._graph))
    empty = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        with torch.cuda.graph(empty, stream=s):
            for _ in range(160):
                bench.trace_mark(4)
    x = torch.empty(64 << 20, device="cuda")
    y = torch.empty_like(x)

    def bw():  # 12 launches of 512 MB traffic each (~0.1 ms apiece at 5-6 TB/s)
        for _ in range(12):
            y.copy_(x)

    xs, ys = x[:16 << 20], y[:16 << 20]

    def bw4():  # the same launches at a quarter of the bytes
        for _ in range(12):
            ys.copy_(xs)

    from sdreamer import _native as nat
    from sdreamer import kernels as K
    stamps = torch.zeros(2 * 512, dtype=torch.int64, device="cuda")
    sink = torch.empty(512, device="cuda")

    def mfma():  # 512 workgroups of dependent f32 MFMA chains, no memory traffic
        nat.call("sd_clock_probe", stamps.data_ptr(), sink.data_ptr(), 512, 60000, K.stream())

    fillers = (("empty x160", empty.replay), ("copies 6 GB", bw), ("copies 1.5 GB", bw4), ("MFMA-only", mfma))
    for crit, fill in (("S1", "M1"), ("M2a", "S2")):
        line = f"{crit}: alone {contended(G[crit].replay, None, reps):7.3f} ms | beside {fill} " \
               f"{contended(G[crit].replay, G[fill].replay, reps):7.3f}"
        for nm, f in fillers:
            line += f" | beside {nm} {contended(G[crit].replay, f, reps):7.3f}"
        print(line)
    line = f"filler alone: M1 {contended(G['M1'].replay, None, reps):.3f} S2 {contended(G['S2'].replay, None, reps):.3f}"
    for nm, f in fillers:
        line += f" | {nm} {contended(f, None, reps):.3f}"
    print(line + " ms")


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    only = sys.argv[2].split(",") if len(sys.argv) > 2 else None
    from sdreamer import networks
    from sdreamer.config import load_config
    from sdreamer.dreamer import Dreamer
    cfg = load_config("dmc/cnn", ["device=cuda:0", "model.compile=False"])
    torch.manual_seed(0)
    agent = Dreamer(cfg.model, bench._Spaces({"image": bench._Sp((64, 64, 3))}), bench._Sp((6,)))
    buf = bench.synth_buffer(cfg, torch.device("cuda", 0), 0)
    for _ in range(4):
        agent.update(buf)
    torch.cuda.synchronize()
    if only == ["contention"]:
        contention(agent, reps)
        return
    names = ("S0", "P", "S1", "M1", "R", "M2a", "S3", "M2b", "S4", "M2c", "M2d", "S2", "M3")
    for nm, g in zip(names, agent._graph):
        if g is not None and (only is None or nm in only):
            if only is not None:  # kernel-trace window around this phase's timed replays (tools/phase_trace.sh)
                g.replay()
                bench.trace_mark(1)
            print(f"phase {nm:4s} alone: {timed(g.replay, reps):8.3f} ms")
            if only is not None:
                bench.trace_mark(2)
    if only is not None:
        return
    r = agent.rssm
    N, H1 = 1024, 16
    g = torch.Generator(device="cuda").manual_seed(1)
    feats = torch.randn(H1, N, r.feat_size, device="cuda", generator=g)
    with torch.no_grad():
        for fused in (True, False):
            networks.FUSED_HEADS = fused
            print(f"heads + returns (fused heads {fused}): {timed(lambda: agent._heads_returns(feats), reps):8.3f} ms")
            heads = (agent.reward, agent.cont, agent.value, agent._slow_value)
            flat = feats.reshape(H1 * N, -1)
            print(f"  heads_nograd only: {timed(lambda: networks.heads_nograd(heads, flat, True), reps):8.3f} ms")
        networks.FUSED_HEADS = True
        from sdreamer import kernels as K
        w = torch.stack([h.mlp._mods[0][0].weight for h in heads])
        b = torch.stack([h.mlp._mods[0][0].bias for h in heads])
        M, F = flat.shape
        h0 = torch.empty(4, M, 256, device="cuda")
        p0 = torch.empty(4, 4, M, device="cuda")
        print(f"  layer-0 batched GEMM (mlp kernel, partials): "
              f"{timed(lambda: K.mlp_layer(flat.expand(4, M, F), w, h0, bias=b, part_out=p0), reps) * 1e3:8.1f} us")
        print(f"  layer-0 batched GEMM (gemm3): "
              f"{timed(lambda: K.gemm(flat.expand(4, M, F), w.transpose(1, 2), h0, bias=b, fast=True), reps) * 1e3:8.1f} us")


if __name__ == "__main__":
    main()
