"""Census of the ATen (non-HIP-extension) operations one eager update issues at the bench shape, per update phase and
calling site: every aten op on device tensors that is not a view / allocation (those launch no kernel) is recorded
under a TorchDispatchMode with the innermost sdreamer frame that issued it. Phase = the agent's last _mark label.
Usage: python tools/aten_census.py [graphs]"""
import collections
import os
import sys
import traceback

os.environ.setdefault("SDREAMER_SIDE_STREAM", "0")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "safe-dreamer_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from torch.utils._python_dispatch import TorchDispatchMode  # noqa: E402

import bench  # noqa: E402

NO_KERNEL = {"view", "_unsafe_view", "_reshape_alias", "reshape", "t", "transpose", "permute", "expand", "as_strided",
             "detach", "alias", "slice", "select", "unsqueeze", "squeeze", "split", "unbind", "empty", "empty_like",
             "empty_strided", "new_empty", "new_empty_strided", "narrow", "chunk", "split_with_sizes", "lift_fresh",
             "_local_scalar_dense", "is_nonzero", "item", "numel", "size", "stride", "dim", "is_same_size",
             "_has_compatible_shallow_copy_type", "set_", "resize_", "view_as", "unfold", "diagonal", "movedim",
             "record_stream", "_to_copy_nocopy"}


def site():
    """the two innermost sdreamer frames (file:function:line < caller), or "autograd" for backward-engine ops"""
    got = []
    for fr in reversed(traceback.extract_stack()[:-3]):
        f = fr.filename
        if "sdreamer" in f and not f.endswith(("_native.py",)):
            got.append(f"{os.path.basename(f)}:{fr.name}:{fr.lineno}")
            if len(got) == 2:
                break
    return " < ".join(got) if got else "autograd"


class Census(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.phase = "start"
        self.recs = collections.Counter()

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        name = func.overloadpacket.__name__
        out = func(*args, **(kwargs or {}))
        if name not in NO_KERNEL:
            dev = any(isinstance(a, torch.Tensor) and a.is_cuda for a in list(args) + list((kwargs or {}).values()))
            if dev or name in ("zeros", "ones", "full", "zeros_like", "ones_like", "full_like", "arange", "scalar_tensor"):
                a0 = args[0] if args and isinstance(args[0], torch.Tensor) else None
                shp = f" {tuple(a0.shape)}/{a0.stride()}" if a0 is not None and name in ("clone", "copy_", "_to_copy",
                                                                                       "contiguous") else ""
                self.recs[(self.phase, name + shp, site())] += 1
        return out


def main():
    from sdreamer.config import load_config
    from sdreamer.dreamer import Dreamer
    cfg = load_config("dmc/cnn", ["device=cuda:0", "model.compile=False"])
    torch.manual_seed(0)
    agent = Dreamer(cfg.model, bench._Spaces({"image": bench._Sp((64, 64, 3))}), bench._Sp((6,)))
    graphs = len(sys.argv) > 1 and sys.argv[1] == "graphs"
    # graphs: the census runs over the update that captures the phase graphs (every op then recorded is one the
    # graph replays in the timed window) plus the eager glue around them
    agent.use_graphs = graphs
    buf = bench.synth_buffer(cfg, torch.device("cuda", 0), 0)
    for _ in range(2):
        agent.update(buf)
    torch.cuda.synchronize()
    c = Census()
    orig = agent._mark

    def mark(name):
        c.phase = name
        return orig(name)
    agent._mark = mark
    with c:
        agent.update(buf)
    torch.cuda.synchronize()
    per = collections.Counter()
    for (ph, _, _), n in c.recs.items():
        per[ph] += n
    print(f"{sum(c.recs.values())} ATen ops in one {'graph-capturing' if graphs else 'eager'} update (phase = the "
          f"agent's last mark before the op)")
    for ph, n in per.items():
        print(f"\n## after mark '{ph}': {n}")
        for (p2, name, s), m in sorted(c.recs.items(), key=lambda kv: kv[0][2]):
            if p2 == ph:
                print(f"  {m:3d} x {name:28s} {s}")


if __name__ == "__main__":
    main()
