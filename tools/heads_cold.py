"""The imagined heads' first layer (four 256 x 2560 weights over 16384 rows, one split-bf16 MLP launch) timed warm
(back to back) and cold (a 1 GiB buffer rewritten between launches, so neither operand is in L2 or the Infinity
Cache), HIP events around the GEMM only, median of 20. Asks whether the 440 us it takes inside the update against
~270 us re-launched alone is cache state. GPU box: python tools/heads_cold.py"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "safe-dreamer_amd"))
import torch  # noqa: E402

from sdreamer import kernels as k  # noqa: E402


def main():
    M, K, U = 16384, 2560, 256
    x = torch.randn(M, K, device="cuda")
    ws = [torch.randn(U, K, device="cuda") * 0.02 for _ in range(4)]
    bs = [torch.randn(U, device="cuda") for _ in range(4)]
    out = torch.empty(4, M, U, device="cuda")
    pout = torch.empty(4, U // 64, M, device="cuda")
    junk = torch.empty(256 * 1024 * 1024, device="cuda")  # 1 GiB
    run = lambda: k.mlp_layer(x[None].expand(4, M, K), ws, out, bias=bs, part_out=pout)  # noqa: E731
    for cold in (False, True):
        for _ in range(3):
            run()
        ts = []
        for _ in range(20):
            if cold:
                junk.fill_(1.0)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            run()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        ts.sort()
        print(f"heads L0 mlp 4x16384x256x2560 {'cold' if cold else 'warm'}: median {ts[10]:.1f} us "
              f"(min {ts[0]:.1f}, max {ts[-1]:.1f})", flush=True)


if __name__ == "__main__":
    main()
