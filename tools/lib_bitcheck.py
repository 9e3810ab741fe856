"""Bit-identity check between two builds of libsdhip.so (A/B aid): computes the split-bf16 conv bwd-weight /
bwd-data, the fused imagination of the bench agent (random init, seed 0) and the parameters after two eager updates
of that agent on the bench's synthetic buffer, on fixed inputs, with the library SDHIP_LIB points at, and saves them to
argv[1]; `python tools/lib_bitcheck.py cmp a.npz b.npz` reports whether every array is bit-identical."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "safe-dreamer_amd"), os.path.join(ROOT, "tests")]


def run(out):
    import torch
    from sdreamer import kernels as K
    res = {}
    for ci, co, hw, nb in [(32, 48, 32, 64), (48, 64, 16, 64), (64, 64, 8, 64), (4, 32, 64, 8)]:
        g = torch.Generator().manual_seed(ci * 7 + co)
        x = (torch.rand(nb, hw, hw, ci, generator=g) - 0.5).cuda()
        dy = torch.randn(nb, hw, hw, co, generator=g).cuda()
        w = (torch.randn(co, 5, 5, ci, generator=g) / (ci * 25) ** 0.5).cuda()
        res[f"dw_{ci}_{co}"] = K.conv2d_wgrad(x, dy, 5, 5, fast=True).cpu().numpy()
        res[f"dx_{ci}_{co}"] = K.conv2d_dgrad(dy, w, fast=True).cpu().numpy()
    import bench
    from sdreamer.config import load_config
    from sdreamer.dreamer import Dreamer
    cfg = load_config("dmc/cnn", ["device=cuda:0", "model.compile=False"])
    torch.manual_seed(0)
    ag = Dreamer(cfg.model, bench._Spaces({"image": bench._Sp((64, 64, 3))}), bench._Sp((6,)))
    g = torch.Generator().manual_seed(3)
    N, S, Kd, D = 1024, ag.rssm._stoch, ag.rssm._discrete, ag.rssm._deter
    stoch = torch.nn.functional.one_hot(torch.randint(0, Kd, (N, S), generator=g), Kd).float().cuda()
    deter = (0.5 * torch.randn(N, D, generator=g)).cuda()
    f, a = ag._imagine_tm((stoch, deter), 16, seed=77, row_offset=0)
    torch.cuda.synchronize()
    res["imag_feat"], res["imag_act"] = f.cpu().numpy(), a.cpu().numpy()
    # two eager updates (scan, encoder, heads, imagination, optimizer) on the bench's synthetic buffer
    L = int(cfg.batch_length)
    buf = bench.synth_buffer(cfg, torch.device("cuda", 0), 0, T=max(160, 2 * (L + 1)), A=6, discrete=False)
    for _ in range(2):
        ag.update(buf)
    torch.cuda.synchronize()
    res["update_params"] = ag._optimizer.arena.data.detach().cpu().numpy()
    np.savez(out, **res)


def cmp(a, b):
    za, zb = np.load(a), np.load(b)
    ok = True
    for k in za.files:
        same = np.array_equal(za[k].view(np.uint32), zb[k].view(np.uint32))
        print(f"{k}: {'bit-identical' if same else 'DIFFERENT max abs %.3g' % np.abs(za[k] - zb[k]).max()}")
        ok &= same
    print("ALL BIT-IDENTICAL" if ok else "MISMATCH")
    return 0 if ok else 1


if __name__ == "__main__":
    if sys.argv[1] == "cmp":
        sys.exit(cmp(sys.argv[2], sys.argv[3]))
    run(sys.argv[1])
