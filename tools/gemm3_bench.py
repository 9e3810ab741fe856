"""f32 vs split-bf16 GEMM timing on the update's shapes (HIP events, median of 20). Usage: python tools/gemm3_bench.py"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "safe-dreamer_amd"))
import torch  # noqa: E402

from sdreamer import kernels as k  # noqa: E402

SHAPES = [  # (label, M, N, K, a_kcontig, b_kcontig)
    ("heads L0 fwd 16384x256x2560", 16384, 256, 2560, True, True),
    ("actor L0 dW 256x2560x15360", 256, 2560, 15360, False, False),
    ("actor L0 dX 15360x2560x256", 15360, 2560, 256, True, False),
    ("value L1 dW 256x256x15360", 256, 256, 15360, False, False),
    ("barlow c 1024x1024x1024", 1024, 1024, 1024, False, False),
    ("square 4096^3", 4096, 4096, 4096, True, True),
]


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(n):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts.sort()
    return ts[len(ts) // 2]


for label, M, N, K, ak, bk in SHAPES:
    a = torch.randn(M, K, device="cuda") if ak else torch.randn(K, M, device="cuda").t()
    b = torch.randn(N, K, device="cuda").t() if bk else torch.randn(K, N, device="cuda")
    out = torch.empty(M, N, device="cuda")
    fl = 2.0 * M * N * K
    t32 = timeit(lambda: k.gemm(a, b, out))
    t3 = timeit(lambda: k.gemm(a, b, out, fast=True))
    print(f"{label:34s} f32 {t32*1e3:8.1f} us {fl/t32/1e9:6.1f} TF | bf16x3 {t3*1e3:8.1f} us {fl/t3/1e9:6.1f} TF"
          f" | x{t32/t3:4.2f}", flush=True)

# the update's own launches: the four imagined heads' first layer in one MLP launch (A broadcast, per-entry weights,
# row partials out), and the weight + bias gradient of the actor / value layer 0 (K-split by the default heuristic)
M, K, U = 16384, 2560, 256
x = torch.randn(M, K, device="cuda")
ws = [torch.randn(U, K, device="cuda") * 0.02 for _ in range(4)]
bs = [torch.randn(U, device="cuda") for _ in range(4)]
out = torch.empty(4, M, U, device="cuda")
pout = torch.empty(4, U // 64, M, device="cuda")
t = timeit(lambda: k.mlp_layer(x[None].expand(4, M, K), ws, out, bias=bs, part_out=pout))
print(f"{'heads L0 mlp 4x16384x256x2560':34s} bf16x3 {t*1e3:8.1f} us {4*2.0*M*U*K/t/1e9:6.1f} TF", flush=True)
R, O, I = 15360, 256, 2560
dy, xx = torch.randn(R, O, device="cuda"), torch.randn(R, I, device="cuda")
dw, db = torch.zeros(O, I, device="cuda"), torch.zeros(O, device="cuda")
t = timeit(lambda: k.wgrad(dy, xx, dw, db))
print(f"{'wgrad+bias 256x2560x15360':34s} bf16x3 {t*1e3:8.1f} us {2.0*R*O*I/t/1e9:6.1f} TF", flush=True)
