"""Encoder stage-1 forward (4 -> 32 channels at 64 x 64, conv_fwd_direct_pool_c4) at the bench's B*L = 1024 images,
per grid shape (GPU box, measurement aid): SDHIP_C4_TPW = tiles per workgroup (16 = the round-5 grid, 2048
workgroups), SDHIP_C4_OCC = resident workgroups per CU the default grid is sized for (one round of them). Every
variant runs the same products per tile, so the outputs must be bit-identical to the round-5 grid's; prints the
median us of back-to-back launches.
  python tools/c4_time.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "safe-dreamer_amd"))
import torch  # noqa: E402

from sdreamer import kernels as K  # noqa: E402


def timeit(fn, n=20):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(n):
            fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e) / n * 1e3)
    return sorted(ts)[2]


def main():
    g = torch.Generator().manual_seed(0)
    x = (torch.rand(1024, 64, 64, 4, generator=g) - 0.5).cuda()
    w = (torch.randn(32, 5, 5, 4, generator=g) / 100 ** 0.5).cuda()
    b = torch.zeros(32).cuda()
    nw = torch.ones(32).cuda()
    ref = None
    flop = 2 * 1024 * 64 * 64 * 32 * 25 * 4
    for tpw, occ in [("16", ""), ("8", ""), ("4", ""), ("", "3"), ("", "4"), ("", "2"), ("16", "")]:
        for k, v in (("SDHIP_C4_TPW", tpw), ("SDHIP_C4_OCC", occ)):
            if v:
                os.environ[k] = v
            else:
                os.environ.pop(k, None)
        out = K.conv2d_fwd_pool(x, w, b, nw)
        if ref is None:
            ref = [t.clone() for t in out]
        same = all(torch.equal(a, r) for a, r in zip(out, ref))
        us = timeit(lambda: K.conv2d_fwd_pool(x, w, b, nw))
        print(f"TPW={tpw or 'auto'} OCC={occ or 'default'}: {us:.1f} us  {flop / us / 1e6:.1f} TF/s  "
              f"bit-identical={same}", flush=True)
        assert same


if __name__ == "__main__":
    main()
