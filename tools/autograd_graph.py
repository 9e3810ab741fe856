"""Print the autograd graph behind the world-model total of one eager update (GPU box, diagnostics for the ATen
census): every node type with its count, and the nodes that are not the library's own Functions.
  python tools/autograd_graph.py"""
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "safe-dreamer_amd")]
os.environ.setdefault("SDREAMER_SIDE_STREAM", "0")
import torch  # noqa: E402

import bench  # noqa: E402


def walk(root):
    seen, order, stack = set(), [], [(root, 0)]
    while stack:
        fn, depth = stack.pop()
        if fn is None or fn in seen:
            continue
        seen.add(fn)
        order.append((fn, depth))
        for nxt, _ in fn.next_functions:
            stack.append((nxt, depth + 1))
    return order


def main():
    from sdreamer.config import load_config
    from sdreamer.dreamer import Dreamer
    cfg = load_config("dmc/cnn", ["device=cuda:0", "model.compile=False"])
    torch.manual_seed(0)
    ag = Dreamer(cfg.model, bench._Spaces({"image": bench._Sp((64, 64, 3))}), bench._Sp((6,)))
    ag.use_graphs = False
    buf = bench.synth_buffer(cfg, torch.device("cuda", 0), 0)
    orig = torch.autograd.backward

    def spy(tensors, grad_tensors=None, *a, **kw):
        ts = tensors if isinstance(tensors, (list, tuple)) else [tensors]
        for t in ts:
            if t.grad_fn is None:
                continue
            nodes = walk(t.grad_fn)
            cnt = collections.Counter(type(n).__name__ for n, _ in nodes)
            print(f"backward from {type(t.grad_fn).__name__} {tuple(t.shape)}: {len(nodes)} nodes")
            for name, c in sorted(cnt.items(), key=lambda kv: -kv[1]):
                print(f"   {c:3d} x {name}")
            for n, d in nodes:
                nm = type(n).__name__
                if nm.endswith("Backward") and not nm.startswith(("LinearFn", "RmsSiluFn")) or nm in ("AccumulateGrad",):
                    v = getattr(n, "variable", None)
                    print(f"      depth {d:2d} {nm} {tuple(v.shape) if v is not None else ''}")
        return orig(tensors, grad_tensors, *a, **kw)

    for _ in range(2):
        ag.update(buf)
    torch.autograd.backward = spy
    ag.update(buf)
    torch.autograd.backward = orig
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
