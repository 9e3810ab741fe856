"""Census of the ATen (non-HIP-extension) operations one eager update issues at the bench shape, per update phase and
calling site: every aten op on device tensors that is not a view / allocation (those launch no kernel) is recorded
under a TorchDispatchMode with the innermost sdreamer frame that issued it. Phase = the agent's last _mark label.
Usage: python tools/aten_census.py"""
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
    for fr in reversed(traceback.extract_stack()[:-3]):
        f = fr.filename
        if "sdreamer" in f and not f.endswith(("_native.py",)):
            return f"{os.path.basename(f)}:{fr.name}:{fr.lineno}"
    return "?"


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
                self.recs[(self.phase, name, site())] += 1
        return out


def main():
    from sdreamer.config import load_config
    from sdreamer.dreamer import Dreamer
    cfg = load_config("dmc/cnn", ["device=cuda:0", "model.compile=False"])
    torch.manual_seed(0)
    agent = Dreamer(cfg.model, bench._Spaces({"image": bench._Sp((64, 64, 3))}), bench._Sp((6,)))
    agent.use_graphs = False
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
    print(f"{sum(c.recs.values())} ATen ops in one eager update (phase = the agent's last mark before the op)")
    for ph, n in per.items():
        print(f"\n## after mark '{ph}': {n}")
        for (p2, name, s), m in sorted(c.recs.items(), key=lambda kv: kv[0][2]):
            if p2 == ph:
                print(f"  {m:3d} x {name:28s} {s}")


if __name__ == "__main__":
    main()
