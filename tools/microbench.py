"""Kernel microbenchmarks on the GPU (HIP events): conv vs dense GEMM of the same shape, GEMM tile variants."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "safe-dreamer_amd"))
import torch  # noqa: E402

from sdreamer import kernels as K  # noqa: E402


def timeit(fn, n=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3  # us


def report(name, flops, us):
    print(f"{name:60s} {us:9.1f} us  {flops / us / 1e6:7.1f} TF/s", flush=True)


def main():
    dev = "cuda"
    torch.manual_seed(0)
    # encoder conv2: 1024 x 32x32x32 -> 48, 5x5
    x = torch.randn(1024, 32, 32, 32, device=dev)
    w = torch.randn(48, 5, 5, 32, device=dev) * 0.05
    b = torch.randn(48, device=dev)
    fl = 2.0 * 1024 * 32 * 32 * 48 * 800
    report("conv2 fwd (im2col implicit GEMM)", fl, timeit(lambda: K.conv2d_fwd(x, w, b)))
    A = torch.randn(1024 * 32 * 32, 800, device=dev)
    W = torch.randn(48, 800, device=dev)
    out = torch.empty(A.shape[0], 48, device=dev)
    for tile in (0, 1, 3):
        report(f"dense gemm 1M x 48 x 800 tile {tile}", fl, timeit(lambda: K.gemm(A, W.t(), out, tile=tile)))
    W64 = torch.randn(64, 800, device=dev)
    out64 = torch.empty(A.shape[0], 64, device=dev)
    report("dense gemm 1M x 64 x 800 tile 3", 2.0 * A.shape[0] * 64 * 800,
           timeit(lambda: K.gemm(A, W64.t(), out64, tile=3)))
    # big square
    a = torch.randn(4096, 4096, device=dev)
    bb = torch.randn(4096, 4096, device=dev)
    o = torch.empty(4096, 4096, device=dev)
    for tile in (0, 1, 3):
        report(f"dense gemm 4096^3 tile {tile}", 2.0 * 4096 ** 3, timeit(lambda: K.gemm(a, bb.t(), o, tile=tile), 5))
    # imagination-like
    xi = torch.randn(1024, 2048, device=dev)
    wi = torch.randn(256, 2048, device=dev)
    oi = torch.empty(1024, 256, device=dev)
    for ks in (1, 2, 4, 8):
        for tile in (0, 1, 3):
            report(f"gemm 1024x256x2048 tile {tile} ks {ks}", 2.0 * 1024 * 256 * 2048,
                   timeit(lambda: K.gemm(xi, wi.t(), oi, tile=tile, ksplit=ks)))
    # heads-like
    xh = torch.randn(16384, 2560, device=dev)
    wh = torch.randn(256, 2560, device=dev)
    oh = torch.empty(16384, 256, device=dev)
    for tile in (0, 1, 3):
        report(f"gemm 16384x256x2560 tile {tile}", 2.0 * 16384 * 256 * 2560, timeit(lambda: K.gemm(xh, wh.t(), oh, tile=tile)))
    # wgrad conv2
    dy = torch.randn(1024, 32, 32, 48, device=dev)
    report("conv2 wgrad", 2.0 * 1024 * 32 * 32 * 48 * 801, timeit(lambda: K.conv2d_wgrad(x, dy, 5, 5)))
    # m16 GEMV
    xs = torch.randn(16, 2048, device=dev)
    os_ = torch.empty(16, 256, device=dev)
    report("m16 16x256x2048", 2.0 * 16 * 256 * 2048, timeit(lambda: K.gemm(xs, wi.t(), os_)))
    ws = torch.randn(2048, 768, device=dev)
    xc = torch.randn(16, 768, device=dev)
    oc = torch.empty(16, 2048, device=dev)
    report("m16 16x2048x768", 2.0 * 16 * 2048 * 768, timeit(lambda: K.gemm(xc, ws.t(), oc)))


if __name__ == "__main__":
    main()
