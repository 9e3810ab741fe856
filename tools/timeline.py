"""Two-stream timeline of one graph-replayed update at the bench shape from device timestamps (SDREAMER_MARKS=1,
kernels.Marks): prints each phase boundary in microseconds since the update's first mark. Usage:
python tools/timeline.py [updates] [config (bench.WORKLOADS)] [per-GPU batch]"""
import os
import sys

os.environ["SDREAMER_MARKS"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "safe-dreamer_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    name = sys.argv[2] if len(sys.argv) > 2 else "dmc/cnn"
    from sdreamer.config import load_config
    from sdreamer.dreamer import Dreamer
    ovr = ["device=cuda:0", "model.compile=False"] + ([f"batch_size={sys.argv[3]}"] if len(sys.argv) > 3 else [])
    cfg = load_config(name, ovr)
    A, discrete, _ = bench.WORKLOADS[name]
    act = bench._Sp((A,))
    if discrete:
        act.discrete = True
    torch.manual_seed(0)
    agent = Dreamer(cfg.model, bench._Spaces({"image": bench._Sp((64, 64, 3))}), act)
    L = int(cfg.batch_length)
    buf = bench.synth_buffer(cfg, torch.device("cuda", 0), 0, T=max(160, 2 * (L + 1)), A=A, discrete=discrete)
    for _ in range(n):
        agent.update(buf)
    torch.cuda.synchronize()
    rows = agent.marks.report()
    prev = {}
    print(f"side stream: {agent.use_side_stream}, graphs: {agent._graph is not None}")
    for tag, us in rows:
        lane = tag.split(":")[0] if ":" in tag else "main"
        d = us - prev.get(lane, 0.0)
        prev[lane] = us
        print(f"{us:9.1f} us  {lane:5s} {tag:24s} (+{d:7.1f})")


if __name__ == "__main__":
    main()
