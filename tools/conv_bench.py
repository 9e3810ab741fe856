"""Per-layer timing of the walker encoder convolutions (fwd, bwd-data, bwd-weight) at B*L = 1024 images."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "safe-dreamer_amd"))
import torch  # noqa: E402

from sdreamer import kernels as K  # noqa: E402


def timeit(fn, n=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


def main():
    Nb = 1024
    layers = [(64, 4, 32), (32, 32, 48), (16, 48, 64), (8, 64, 64)]
    if len(sys.argv) > 1:
        layers = layers[1:]  # (H, Ci, Co); layer 1 padded to 4 channels
    tot = {}
    for H, Ci, Co in layers:
        x = torch.randn(Nb, H, H, Ci, device="cuda")
        w = torch.randn(Co, 5, 5, Ci, device="cuda") * 0.05
        b = torch.randn(Co, device="cuda")
        dy = torch.randn(Nb, H, H, Co, device="cuda")
        fl = 2.0 * Nb * H * H * Co * 25 * Ci
        wf = K.conv_flip_weight(w)
        nw = torch.ones(Co, device="cuda")
        ws = K.conv_split_weight(wf)
        K.set_flip_cache([w])  # the update's state: flipped + split weights cached ahead of the backward

        def fpool6():
            K.CONV6 = "1"
            try:
                return K.conv2d_fwd_pool(x, w, b, nw)
            finally:
                K.CONV6 = ""

        del ws
        for name, fn in (("fwd", lambda: K.conv2d_fwd(x, w, b)), ("fpool", lambda: K.conv2d_fwd_pool(x, w, b, nw)),
                         ("fpool6", fpool6),
                         ("dgrad", lambda: K.conv2d_fwd(dy, wf, None)),
                         ("dgrad3", lambda: K.conv2d_dgrad(dy, w, pad=2, fast=True, direct=False)),
                         ("dgrad3d", lambda: K.conv2d_dgrad(dy, w, pad=2, fast=True)),
                         ("wgrad", lambda: K.conv2d_wgrad(x, dy, 5, 5, fast=False)),
                         ("wgrad3", lambda: K.conv2d_wgrad(x, dy, 5, 5, fast=True))):
            us = timeit(fn)
            tot[name] = tot.get(name, 0) + us
            print(f"H{H:3d} Ci{Ci:3d} Co{Co:3d} {name:6s} {us:9.1f} us {fl / us / 1e6:7.1f} TF/s", flush=True)
    print("totals", {k: round(v, 1) for k, v in tot.items()}, flush=True)


if __name__ == "__main__":
    main()
