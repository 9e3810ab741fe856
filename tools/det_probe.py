"""Determinism probe (GPU box): two agents with identical weights and identical replay buffers, updated in lockstep
(eager or graphed), compared after every update — metrics, every parameter, the LaProp moments and the gradient
arena as the step left it. Prints the first update / tensor that differs.

  python tools/det_probe.py [config] [updates] [graphs: 0|1] [side stream: 0|1]
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "safe-dreamer_amd")]

from bench import WORKLOADS, _Sp, _Spaces, synth_buffer  # noqa: E402


def make(config, graphs, side):
    from sdreamer.config import load_config
    from sdreamer.dreamer import Dreamer
    A, discrete, _ = WORKLOADS[config]
    cfg = load_config(config, ["device=cuda:0", "model.compile=False"])
    torch.manual_seed(0)
    act = _Sp((A,))
    if discrete:
        act.discrete = True
    ag = Dreamer(cfg.model, _Spaces({"image": _Sp((64, 64, 3))}), act)
    ag.use_graphs = graphs
    ag.use_side_stream = side
    L = int(cfg.batch_length)
    buf = synth_buffer(cfg, torch.device("cuda:0"), 0, T=max(160, 2 * (L + 1)), A=A, discrete=discrete)
    return ag, buf


def main():
    config = sys.argv[1] if len(sys.argv) > 1 else "dmc/cnn"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    graphs = bool(int(sys.argv[3])) if len(sys.argv) > 3 else False
    side = bool(int(sys.argv[4])) if len(sys.argv) > 4 else True
    a, ba = make(config, graphs, side)
    b, bb = make(config, graphs, side)
    for u in range(n):
        ma = {k: float(v) for k, v in a.update(ba).items()}
        mb = {k: float(v) for k, v in b.update(bb).items()}
        torch.cuda.synchronize()
        dm = [k for k in ma if ma[k] != mb[k] and not (ma[k] != ma[k] and mb[k] != mb[k])]
        sa, sb = a.state_dict(), b.state_dict()
        dp = [k for k in sa if torch.is_tensor(sa[k]) and not torch.equal(sa[k], sb[k])]
        oa, ob = a._optimizer, b._optimizer
        dv = not torch.equal(oa.exp_avg_sq, ob.exp_avg_sq)
        dmom = not torch.equal(oa.exp_avg, ob.exp_avg)
        dst = [k for k in ("stoch", "deter") if not torch.equal(ba._store[k], bb._store[k])]
        print(f"update {u}: metrics differ {len(dm)} {dm[:6]}; params differ {len(dp)} {dp[:6]}; "
              f"v differs {dv}; m differs {dmom}; storage differs {dst}", flush=True)
        if dp or dm:
            for k in dp[:3]:
                d = (sa[k].double() - sb[k].double()).abs()
                print(f"   {k}: max |diff| {d.max().item():.3g} at {int(d.argmax())}, n diff {(d > 0).sum().item()}")
            if dv:
                d = (oa.exp_avg_sq.double() - ob.exp_avg_sq.double()).abs()
                i = int(d.argmax())
                # which parameter tensor holds the first differing second-moment element
                nz = (d > 0).nonzero()
                first = int(nz[0]) if len(nz) else -1
                offs = oa.arena.offsets
                owner = max(j for j in range(len(offs)) if offs[j] <= first) if first >= 0 else -1
                names = [nm for nm, p in a._named_params.items()]
                print(f"   v: max diff {d.max().item():.3g} at {i}; first diff elem {first} in tensor #{owner} "
                      f"({names[owner] if 0 <= owner < len(names) else '?'}), n diff {len(nz)}")
            break


if __name__ == "__main__":
    main()
