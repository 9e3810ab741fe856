"""Host-side cost of one update at the bench shape: CPU time of agent.update() (no sync; graph replay is
asynchronous), of the graph launch alone, and the synchronized wall time per update."""
import os
import sys
import time

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
    agent = Dreamer(cfg.model, bench._Spaces({"image": bench._Sp((64, 64, 3))}), bench._Sp((6,)))
    buf = bench.synth_buffer(cfg, torch.device("cuda", 0), 0)
    for _ in range(5):
        agent.update(buf)
    torch.cuda.synchronize()
    gs = agent._graph if isinstance(agent._graph, tuple) else (agent._graph,)
    n = 10
    for i, g in enumerate(x for x in gs if x is not None):
        t0 = time.perf_counter()
        for _ in range(n):
            g.replay()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"graph {i} replay(): host {1e3 * (t1 - t0) / n:.3f} ms/launch, back-to-back wall "
              f"{1e3 * (t2 - t0) / n:.3f} ms")
    t0 = time.perf_counter()
    for _ in range(n):
        agent.update(buf)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"agent.update(): host {1e3 * (t1 - t0) / n:.3f} ms/update, wall {1e3 * (t2 - t0) / n:.3f} ms/update")


if __name__ == "__main__":
    main()
