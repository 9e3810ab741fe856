"""Time one sd_gemm_bf16x3_mlp launch at the imagined heads' first-layer shape (dmc/cnn: M = 16 x 1024 rows,
K = feat 2560, four 256-wide heads on one input, row partials out), alone on an idle GPU, with HIP events.
Usage: python tools/mlp_bench.py [M] [K] [reps]  (SDHIP_LIB selects the library build)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "safe-dreamer_amd"))
import torch  # noqa: E402


def main():
    from sdreamer import kernels as kern
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 2560
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    n, N = 4, 256
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(M, K, device="cuda", generator=g)
    ws = [torch.randn(N, K, device="cuda", generator=g) / K ** 0.5 for _ in range(n)]
    bs = [torch.randn(N, device="cuda", generator=g) for _ in range(n)]
    out = torch.empty(n, M, N, device="cuda")
    pout = torch.empty(n, N // 64, M, device="cuda")
    xd = x.expand(n, M, K)
    for _ in range(3):
        assert kern.mlp_layer(xd, ws, out, bias=bs, part_out=pout)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(reps + 1)]
    ev[0].record()
    for i in range(reps):
        kern.mlp_layer(xd, ws, out, bias=bs, part_out=pout)
        ev[i + 1].record()
    torch.cuda.synchronize()
    ts = sorted(ev[i].elapsed_time(ev[i + 1]) * 1e3 for i in range(reps))
    fl = 2.0 * n * M * N * K
    med = ts[len(ts) // 2]
    print(f"mlp_layer M={M} K={K} n={n} N={N}: median {med:.1f} us, min {ts[0]:.1f} us; "
          f"{fl / med / 1e6:.1f} TF/s f32-equivalent = {3 * fl / med / 1e6 / 2500:.3f} of the bf16 dense peak "
          f"(3 MFMA per product)")


if __name__ == "__main__":
    main()
