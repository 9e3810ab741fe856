"""Tile / K-split sweep of the split-bf16 weight-gradient GEMM dW (256 x 2560) = dy^T x over 15360 rows (the actor /
value layer-0 weight gradients of the imagined trajectories), HIP-event median of 20. GPU box.
  python tools/wgrad_sweep.py"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "safe-dreamer_amd"))
import torch  # noqa: E402

from sdreamer import kernels as k  # noqa: E402


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(n):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    return sorted(ts)[n // 2]


def main():
    R, O, I = 15360, 256, 2560
    dy = torch.randn(R, O, device="cuda")
    x = torch.randn(R, I, device="cuda")
    dw = torch.zeros(O, I, device="cuda")
    for tile in (0, 1, 2):
        for ks in (4, 8, 13, 20, 30, 60):
            us = timeit(lambda: k.gemm(dy.t(), x, dw, beta=1.0, fast=True, ksplit=ks, tile=tile))
            print(f"tile {tile} ksplit {ks:3d}: {us:7.1f} us ({2 * R * O * I / us / 1e6:6.1f} TF f32-eq)", flush=True)


if __name__ == "__main__":
    main()
