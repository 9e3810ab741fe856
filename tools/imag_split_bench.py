"""Imagination at the bench shape (N = 1024 start rows, H1 = 16) as one rollout vs row shards rolled out
concurrently on separate streams (each shard its own launch sequence; noise indexed by global row, so the shards
reproduce the full rollout). Prints ms per imagination for 1, 2 and 4 shards."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "safe-dreamer_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
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
    streams = [torch.cuda.Stream() for _ in range(4)]
    main = torch.cuda.current_stream()
    ref = None
    for shards in (1, 2, 4):
        n = N // shards

        def run(seed):
            outs = []
            for k in range(shards):
                st = streams[k]
                st.wait_stream(main)
                with torch.cuda.stream(st):
                    outs.append(agent._imagine_tm((stoch[k * n:(k + 1) * n], deter[k * n:(k + 1) * n]), H1, seed,
                                                  row_offset=k * n))
            for st in streams[:shards]:
                main.wait_stream(st)
            return outs
        with torch.no_grad():
            outs = run(1)
            torch.cuda.synchronize()
            feats = torch.cat([o[0] for o in outs], 1)
            if ref is None:
                ref = feats
            same = torch.equal(feats, ref)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for r in range(reps):
                run(2 + r)
            e.record()
            torch.cuda.synchronize()
        print(f"imagination N={N} H1={H1} as {shards} concurrent shard(s): {s.elapsed_time(e) / reps:.3f} ms "
              f"(bit-identical to 1 shard: {same})", flush=True)


if __name__ == "__main__":
    main()
