"""The imagined heads' input-gradient GEMM (dx = dy W: M = 15,360 imagined rows, N = K = 256, both operands
K-contiguous, split-bf16) alone, per tile shape, HIP-graph timed (GPU box, measurement aid). In the update's trace it
lasts 49-66 us beside the scan backward; this prints what it costs alone.
  python tools/g3_dx_time.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "safe-dreamer_amd"))
import torch  # noqa: E402

from sdreamer import kernels as K  # noqa: E402


def graph_us(fn, reps=20):
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(reps):
                fn()
    ts = []
    for _ in range(5):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3 / reps)
    return sorted(ts)[2]


def main():
    torch.manual_seed(0)
    M, N, Kd = 15360, 256, 256
    dy = torch.randn(M, Kd, device="cuda")
    w = torch.randn(Kd, N, device="cuda") / 16  # layer weight (out = Kd, in = N): dx = dy @ w
    wt = w.t().contiguous()
    out = torch.empty(M, N, device="cuda")
    ref = dy.double() @ w.double()
    for name, b, tile in [("B k-contig, auto tile", wt.t(), -1), ("B k-contig, 64x64", wt.t(), 1),
                          ("B k-contig, 128x128", wt.t(), 0), ("B rows-contig, auto", w, -1)]:
        us = graph_us(lambda: K.gemm(dy, b, out, fast=True, tile=tile))
        err = ((out.double() - ref).abs().max() / ref.abs().max()).item()
        mb = (M * Kd + Kd * N + M * N) * 4 / 1e6
        print(f"{name}: {us:.1f} us  ({mb / us:.2f} TB/s algorithmic, max rel err {err:.1e})", flush=True)


if __name__ == "__main__":
    main()
