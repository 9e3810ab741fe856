"""Tile / K-split sweep of the imagined heads' 256-wide hidden-layer GEMMs on the split-bf16 kernel (GPU box,
measurement aid): (a) the weight gradient dW (256 x 256) = dy^T x over 15360 rows, (b) the input gradient
dx (15360 x 256) = dy W. HIP-event median of 20 launches each.
  python tools/g3_small_sweep.py"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "safe-dreamer_amd"))
import torch  # noqa: E402

from sdreamer import kernels as k  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from wgrad_sweep import timeit  # noqa: E402


def main():
    R, O = 15360, 256
    dy = torch.randn(R, O, device="cuda")
    x = torch.randn(R, O, device="cuda")
    w = torch.randn(O, O, device="cuda")
    dw = torch.zeros(O, O, device="cuda")
    dx = torch.zeros(R, O, device="cuda")
    fl = 2 * R * O * O
    us = timeit(lambda: k.gemm(dy.t(), x, dw, beta=1.0, fast=True))
    print(f"(a) dW default: {us:7.1f} us ({fl / us / 1e6:6.1f} TF f32-eq)", flush=True)
    for tile in (0, 1):
        for ks in (4, 8, 15, 16, 20, 30, 32, 40, 48, 60, 96, 120):
            us = timeit(lambda: k.gemm(dy.t(), x, dw, beta=1.0, fast=True, ksplit=ks, tile=tile))
            print(f"(a) dW tile {tile} ksplit {ks:3d}: {us:7.1f} us ({fl / us / 1e6:6.1f} TF f32-eq)", flush=True)
    us = timeit(lambda: k.gemm(dy, w, dx, fast=True))
    print(f"(b) dx default: {us:7.1f} us ({fl / us / 1e6:6.1f} TF f32-eq)", flush=True)
    for tile in (0, 1):
        for ks in (1, 2, 4):
            us = timeit(lambda: k.gemm(dy, w, dx, fast=True, ksplit=ks, tile=tile))
            print(f"(b) dx tile {tile} ksplit {ks}: {us:7.1f} us ({fl / us / 1e6:6.1f} TF f32-eq)", flush=True)


if __name__ == "__main__":
    main()
