"""Policy latency: Dreamer.act per env step, eager vs the replayed graph (Dreamer.policy_graph),
walker vision config, B environments. Usage: python tools/act_bench.py [B]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "safe-dreamer_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    from sdreamer.config import load_config
    from sdreamer.dreamer import Dreamer
    cfg = load_config("dmc/cnn", ["device=cuda:0", "model.compile=False"])
    torch.manual_seed(0)
    ag = Dreamer(cfg.model, bench._Spaces({"image": bench._Sp((64, 64, 3))}), bench._Sp((6,)))
    obs = {"image": torch.randint(0, 256, (B, 64, 64, 3), dtype=torch.uint8, device="cuda"),
           "is_first": torch.zeros(B, dtype=torch.bool, device="cuda")}
    state = ag.get_initial_state(B)
    policy = ag.policy_graph(B, obs)
    for name, fn in (("eager", lambda s: ag.act(obs, s)), ("graph", lambda s: policy(obs, s))):
        s = state
        for _ in range(5):
            _, s = fn(s)
        torch.cuda.synchronize()
        n = 200
        t0 = time.perf_counter()
        for _ in range(n):
            a, s = fn(s)
            a.cpu()  # an env step consumes the action on the host
        dt = (time.perf_counter() - t0) / n
        print(f"act B={B} {name}: {dt * 1e6:.1f} us per env step (incl. action device->host)", flush=True)


if __name__ == "__main__":
    main()
