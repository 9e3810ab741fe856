"""Encoder stage forward, per kernel variant, at the bench's B*L = 1024 images (GPU box, measurement aid):
exact f32 (sd_conv2d_fwd_pool), bf16x6 per-lane weight (SDHIP_CONV6_RING=0) and bf16x6 LDS ring, for the 32 -> 48
stage at 32 x 32 and the 48 -> 64 stage at 16 x 16; the ring kernel one tile per workgroup (with / without the
fragment pipeline) and with its default multi-tile workgroups (SDHIP_CONV6_TPW). Prints median us of back-to-back launches.
  python tools/conv6_time.py"""
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
    for hw, ci, co in [(32, 32, 48), (16, 48, 64)]:
        x = (torch.rand(1024, hw, hw, ci, generator=g) - 0.5).cuda()
        w = (torch.randn(co, 5, 5, ci, generator=g) / (ci * 25) ** 0.5).cuda()
        b = torch.zeros(co).cuda()
        nw = torch.ones(co).cuda()
        res = {}
        for name, c6, ring, pipe, tpw in [("f32", "", "1", "0", ""), ("bf16x6 lane", "1", "0", "0", ""),
                                          ("bf16x6 ring pipe 1 tile", "1", "1", "1", ""),
                                          ("bf16x6 ring MT2 1 tile", "1", "1", "0", "mt2:1"),
                                          ("bf16x6 ring MT2", "1", "1", "0", "mt2:"),
                                          ("bf16x6 ring MT4 prefetch x4", "1", "1", "0", "mt4:4"),
                                          ("bf16x6 ring", "1", "1", "0", "")]:
            K.CONV6 = c6
            os.environ["SDHIP_CONV6_RING"] = ring
            os.environ["SDHIP_CONV6_PIPE"] = pipe
            os.environ.pop("SDHIP_CONV6_MT", None)
            if tpw.startswith("mt"):  # the 32 -> 48 stage's m tiles per wave (the 48 -> 64 stage has 2 either way)
                os.environ["SDHIP_CONV6_MT"] = tpw[2]
                tpw = tpw[4:]
            if tpw:
                os.environ["SDHIP_CONV6_TPW"] = tpw
            else:
                os.environ.pop("SDHIP_CONV6_TPW", None)
            res[name] = timeit(lambda: K.conv2d_fwd_pool(x, w, b, nw))
        flop = 2 * 1024 * hw * hw * co * 25 * ci
        print(f"stage {ci}->{co} at {hw}x{hw}: " + "  ".join(f"{k} {v:.1f} us" for k, v in res.items()) +
              f"  (ring: {flop / res['bf16x6 ring'] / 1e6:.1f} TF f32-equivalent)")


if __name__ == "__main__":
    main()
