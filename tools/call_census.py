"""Per-call census of one eager update at the bench shape: every C-ABI launch (sdreamer/_native.call) timed with HIP
events on the stream it is enqueued on, grouped by entry point + calling site + shape. Single stream
(SDREAMER_SIDE_STREAM=0), no graph, so the times add up to the serial update. Usage: python tools/call_census.py [top]
"""
import collections
import os
import sys
import traceback

os.environ.setdefault("SDREAMER_SIDE_STREAM", "0")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "safe-dreamer_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402


def site():
    for fr in reversed(traceback.extract_stack()[:-3]):
        f = os.path.basename(fr.filename)
        if f not in ("kernels.py", "_native.py", "call_census.py"):
            return f"{f}:{fr.name}:{fr.lineno}"
    return "?"


def shape_of(name, args):
    if name == "sd_gemm_f32":
        d = args[0]._obj  # ctypes.byref(GemmDesc)
        return f"M{d.M} N{d.N} K{d.K} b{d.batch} ak{d.a_kcontig} bk{d.b_kcontig} ks{d.ksplit}"
    return " ".join(str(a) for a in args if isinstance(a, int) and not isinstance(a, bool))[:60]


def main():
    top = int(sys.argv[1]) if len(sys.argv) > 1 else 60
    from sdreamer import _native as nat
    from sdreamer.config import load_config
    from sdreamer.dreamer import Dreamer
    cfg = load_config("dmc/cnn", ["device=cuda:0", "model.compile=False"])
    torch.manual_seed(0)
    agent = Dreamer(cfg.model, bench._Spaces({"image": bench._Sp((64, 64, 3))}), bench._Sp((6,)))
    agent.use_graphs = False
    buf = bench.synth_buffer(cfg, torch.device("cuda", 0), 0)
    for _ in range(2):
        agent.update(buf)
    torch.cuda.synchronize()
    recs = []
    orig = nat.call

    def call(name, *args):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        orig(name, *args)
        e.record()
        recs.append((name, site(), shape_of(name, args), s, e))
    nat.call = call
    s0, e0 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s0.record()
    agent.update(buf)
    e0.record()
    torch.cuda.synchronize()
    nat.call = orig
    total = s0.elapsed_time(e0) * 1e3
    agg = collections.defaultdict(lambda: [0, 0.0])
    for name, st, shp, s, e in recs:
        a = agg[(name, st, shp)]
        a[0] += 1
        a[1] += s.elapsed_time(e) * 1e3
    inside = sum(v[1] for v in agg.values())
    print(f"eager serial update: {total:.0f} us wall, {inside:.0f} us inside {len(recs)} C-ABI calls")
    print("| us | calls | entry | site | shape |")
    print("|---:|---:|---|---|---|")
    for (name, st, shp), (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f"| {t:.0f} | {n} | {name} | {st} | {shp} |")
    byname = collections.defaultdict(float)
    for (name, st, shp), (n, t) in agg.items():
        byname[name] += t
    print("\n| us | entry |\n|---:|---|")
    for name, t in sorted(byname.items(), key=lambda kv: -kv[1]):
        print(f"| {t:.0f} | {name} |")


if __name__ == "__main__":
    main()
