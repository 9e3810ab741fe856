"""Imagination-only driver at the bench shape (walker r2dreamer, N = B*T = 1024 start states, H1 = 16): times the
fused imagination with HIP events, for kernel-level profiling (rocprofv3 --pmc) of csrc/img.hip."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "safe-dreamer_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    from sdreamer.config import load_config
    from sdreamer.dreamer import Dreamer
    cfg = load_config("dmc/cnn", ["device=cuda:0", "model.compile=False"])
    torch.manual_seed(0)
    agent = Dreamer(cfg.model, bench._Spaces({"image": bench._Sp((64, 64, 3))}), bench._Sp((6,)))
    N, S, Kd, D = 1024, agent.rssm._stoch, agent.rssm._discrete, agent.rssm._deter
    g = torch.Generator().manual_seed(0)
    stoch = torch.nn.functional.one_hot(torch.randint(0, Kd, (N, S), generator=g), Kd).float().cuda()
    deter = (0.5 * torch.randn(N, D, generator=g)).cuda()
    H1 = agent.imag_horizon + 1
    with torch.no_grad():
        agent._imagine_tm((stoch, deter), H1, seed=1)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for r in range(reps):
            agent._imagine_tm((stoch, deter), H1, seed=2 + r)
        e.record()
        torch.cuda.synchronize()
    print(f"imagination N={N} H1={H1}: {s.elapsed_time(e) / reps:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
