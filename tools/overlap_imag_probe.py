"""Co-scheduling probe: the posterior scan (latency-bound) alone vs beside imagination on 256-row chunks (what a
scan/imagination pipeline would run concurrently). Usage: python tools/overlap_imag_probe.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "safe-dreamer_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    from sdreamer.config import load_config
    from sdreamer.dreamer import Dreamer
    cfg = load_config("dmc/cnn", ["device=cuda:0", "model.compile=False"])
    torch.manual_seed(0)
    ag = Dreamer(cfg.model, bench._Spaces({"image": bench._Sp((64, 64, 3))}), bench._Sp((6,)))
    B, T = 16, 64
    g = torch.Generator().manual_seed(0)
    img = (torch.randint(0, 256, (B, T, 64, 64, 3), generator=g, dtype=torch.uint8).float() / 255).cuda()
    act = (torch.rand(B, T, 6, generator=g) * 2 - 1).cuda()
    first = torch.zeros(B, T, dtype=torch.bool, device="cuda")
    first[:, 0] = True
    init = (torch.zeros(B, 32, 16, device="cuda"), torch.zeros(B, 2048, device="cuda"))
    with torch.no_grad():
        embed = ag.encoder({"image": img})
    S, Kd, D = ag.rssm._stoch, ag.rssm._discrete, ag.rssm._deter
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    st = torch.nn.functional.one_hot(torch.randint(0, Kd, (rows, S), generator=g), Kd).float().cuda()
    de = (0.5 * torch.randn(rows, D, generator=g)).cuda()

    def scan():
        with torch.no_grad():
            ag.rssm.observe(embed, act, init, first, seed=1)

    def imag():
        with torch.no_grad():
            for _ in range(1024 // rows):
                ag._imagine_tm((st, de), 16, seed=1)

    def timed(fn, stream):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(stream):
            s.record()
            fn()
            e.record()
        return s, e

    a, b = torch.cuda.Stream(), torch.cuda.Stream()
    for _ in range(2):
        scan()
        imag()
    torch.cuda.synchronize()
    s, e = timed(scan, a)
    torch.cuda.synchronize()
    t_scan = s.elapsed_time(e)
    s, e = timed(imag, b)
    torch.cuda.synchronize()
    t_imag = s.elapsed_time(e)
    s2, e2 = timed(imag, b)
    s1, e1 = timed(scan, a)
    torch.cuda.synchronize()
    print(f"rows/chunk {rows}: scan alone {t_scan:.3f} ms, imagination (1024 rows in chunks) alone {t_imag:.3f} ms; "
          f"together: scan {s1.elapsed_time(e1):.3f} ms, imagination {s2.elapsed_time(e2):.3f} ms, "
          f"span {s2.elapsed_time(e1):.3f} ms", flush=True)


if __name__ == "__main__":
    main()
