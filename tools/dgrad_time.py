"""Encoder stage-2 bwd-data (sd_conv2d_dgrad_direct, 48 -> 32 channels at 32 x 32) at the bench's 1024 images, per
tile variant (SDHIP_DGRAD_MT: 4 = 512-pixel tiles of 64-pixel waves, 2 = 128-pixel tiles of 32-pixel waves): median
us of back-to-back launches (GPU box, measurement aid).  python tools/dgrad_time.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "safe-dreamer_amd"), os.path.dirname(os.path.abspath(__file__))]
import torch  # noqa: E402

from conv6_time import timeit  # noqa: E402
from sdreamer import kernels as K  # noqa: E402


def main():
    g = torch.Generator().manual_seed(0)
    w = (torch.randn(48, 5, 5, 32, generator=g) / (32 * 25) ** 0.5).cuda()
    dy = torch.randn(1024, 32, 32, 48, generator=g).cuda()
    ws = K.conv_split_weight(K.conv_flip_weight(w))
    dx = torch.empty(1024, 32, 32, 32, device="cuda")
    fl = 2 * 1024 * 32 * 32 * 48 * 25 * 32
    for mt in ("2", "4"):
        os.environ["SDHIP_DGRAD_MT"] = mt
        us = timeit(lambda: K.nat.call("sd_conv2d_dgrad_direct", K.p(dy), K.p(ws), K.p(dx), 1024, 32, 32, 48, 32, 5, 5,
                                       2, K.stream()))
        print(f"dgrad MT{mt}: {us:.1f} us ({fl / us / 1e6:.1f} TF f32-equivalent)")
    os.environ.pop("SDHIP_DGRAD_MT", None)
    w = (torch.randn(64, 5, 5, 48, generator=g) / (48 * 25) ** 0.5).cuda()  # stage 3: 64 -> 48 at 16 x 16
    dy = torch.randn(1024, 16, 16, 64, generator=g).cuda()
    ws = K.conv_split_weight(K.conv_flip_weight(w))
    dx = torch.empty(1024, 16, 16, 48, device="cuda")
    fl = 2 * 1024 * 16 * 16 * 64 * 25 * 48
    for mt in ("2", "4"):  # (SDHIP_DGRAD3_MT: 4 = whole-image tiles of 64-pixel waves, the default)
        os.environ["SDHIP_DGRAD3_MT"] = mt
        us = timeit(lambda: K.nat.call("sd_conv2d_dgrad_direct", K.p(dy), K.p(ws), K.p(dx), 1024, 16, 16, 64, 48, 5, 5,
                                       2, K.stream()))
        print(f"stage-3 dgrad MT{mt}: {us:.1f} us ({fl / us / 1e6:.1f} TF f32-equivalent)")


if __name__ == "__main__":
    main()
