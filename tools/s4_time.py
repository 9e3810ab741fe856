"""Encoder stage-4 forward (64 -> 64 channels at 8 x 8, conv_fwd16_pool<64>) at the bench's B*L = 1024 images alone
(GPU box, measurement aid): median us of back-to-back launches.
  python tools/s4_time.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "safe-dreamer_amd"))
import torch  # noqa: E402

from sdreamer import kernels as K  # noqa: E402
from c4_time import timeit  # noqa: E402


def main():
    g = torch.Generator().manual_seed(0)
    K.CONV6 = ""
    x = (torch.rand(1024, 8, 8, 64, generator=g) - 0.5).cuda()
    w = (torch.randn(64, 5, 5, 64, generator=g) / 40).cuda()
    b = (0.1 * torch.randn(64, generator=g)).cuda()
    nw = torch.ones(64).cuda()
    us = timeit(lambda: K.conv2d_fwd_pool(x, w, b, nw))
    flop = 2 * 1024 * 64 * 64 * 25 * 64
    print(f"stage 64->64 at 8x8: {us:.1f} us  {flop / us / 1e6:.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
