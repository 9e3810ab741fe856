"""k_hid_areg vs k_hid<true> (SDHIP_KH_NOAREG) on one imagination step: the workspace's hp and ph after step 0
(measurement aid on the GPU box)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), ROOT, os.path.join(ROOT, "safe-dreamer_amd")]
import torch  # noqa: E402
from test_gpu_imagine import _start  # noqa: E402
from test_gpu_dreamer import build_agent  # noqa: E402


def al64(n):
    return (n + 63) // 64 * 64


def main():
    name, N = (sys.argv[1], int(sys.argv[2])) if len(sys.argv) > 2 else ("walker_r2", 192)
    ag, z, spec, obs = build_agent(name)
    stoch, deter = _start(ag, N, 11)
    SK, U, D = ag.rssm.flat_stoch, 256, ag.rssm._deter
    os.environ["SDHIP_KL_NOPRE"] = "1"
    out = {}
    for tag, env in [("areg", None), ("noareg", "SDHIP_KH_NOAREG")]:
        if env:
            os.environ[env] = "1"
        feats = torch.empty(2, N, ag.rssm.feat_size, device="cuda")
        feats[0, :, :SK] = stoch.reshape(N, SK)
        feats[0, :, SK:] = deter
        actions = torch.empty(2, N, ag.act_dim, device="cuda")
        keep = {}
        ag._imagine_fused(feats, actions, 2, 77, 5, keep=keep)
        torch.cuda.synchronize()
        w = keep["work"]
        NU, NP = N * U, N * (U // 16)
        o = 2 * (al64(NU) + al64(NP)) + al64(NU) + 2 * (al64(NU) + al64(NP)) + al64(NU)
        hp = w[o:o + N * D].view(N, D).clone()
        o += al64(N * D)
        ph = w[o:o + (D // 64) * N].view(D // 64, N).clone()
        x0 = w[2 * (al64(NU) + al64(NP)) + al64(NU):][:NU].view(N, U).clone()
        out[tag] = (hp, ph, x0, feats.clone())
        if env:
            del os.environ[env]
    a, b = out["areg"], out["noareg"]
    import numpy as np
    np.savez(os.path.join(ROOT, "gpurun_out", "areg_diff2.npz"), hp=a[0].cpu().numpy(), ph_a=a[1].cpu().numpy(),
             ph_b=b[1].cpu().numpy(), bh=ag.rssm._dyn_hid.bias.detach().cpu().numpy() if hasattr(ag.rssm, "_dyn_hid") else np.zeros(1))
    for k, nm in enumerate(["hp", "ph", "x0p", "feats"]):
        d = (a[k] - b[k]).abs()
        bad = (d > 0).nonzero()
        print(f"{nm}: equal={torch.equal(a[k], b[k])} max {float(d.max()):.3g} n_diff {len(bad)} first {bad[:8].tolist()}")


if __name__ == "__main__":
    main()
