"""Where the imagination of k_hid_areg differs from k_hid<true> (SDHIP_KH_NOAREG) and from the in-loader split
(SDHIP_KH_NOAPRE): first step, stoch / deter part, max |diff| (measurement aid on the GPU box)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), ROOT, os.path.join(ROOT, "safe-dreamer_amd")]
import torch  # noqa: E402
from test_gpu_imagine import _run, _start  # noqa: E402
from test_gpu_dreamer import build_agent  # noqa: E402


def main():
    name, N = (sys.argv[1], int(sys.argv[2])) if len(sys.argv) > 2 else ("walker_r2", 192)
    ag, z, spec, obs = build_agent(name)
    start = _start(ag, N, 11)
    SK = ag.rssm.flat_stoch
    os.environ["SDHIP_KL_NOPRE"] = "1"
    runs = {}
    for tag, env in [("areg", None), ("noareg", "SDHIP_KH_NOAREG"), ("noapre", "SDHIP_KH_NOAPRE")]:
        if env:
            os.environ[env] = "1"
        runs[tag] = _run(ag, start, 6, True)
        if env:
            del os.environ[env]
    for x, y in [("areg", "noareg"), ("areg", "noapre"), ("noareg", "noapre")]:
        fa, fb = runs[x][0], runs[y][0]
        d = (fa - fb).abs()
        steps = [t for t in range(fa.shape[0]) if d[t].max() > 0]
        print(f"{x} vs {y}: equal={torch.equal(fa, fb)} first step {steps[:1]}", end=" ")
        if steps:
            t = steps[0]
            dd = d[t]
            rows = (dd.max(1).values > 0).nonzero().flatten()
            print(f"stoch max {float(dd[:, :SK].max()):.3g} deter max {float(dd[:, SK:].max()):.3g} rows {rows[:10].tolist()}"
                  f" ({len(rows)}) deter cols {(dd[:, SK:].max(0).values > 0).nonzero().flatten()[:10].tolist()}")
        else:
            print()


if __name__ == "__main__":
    main()
