"""Float64 LaProp moments of the golden cases (fixture generator; test infrastructure).

Runs the CPU oracle (oracle/ref_cpu.py: the reference's update restated) in float64 (ref_cpu.DT) over each golden
case's two updates, with the case's weights, batches, initial latents and Philox noise (the inputs the reference forms
in f32 — images / 255, the augmentation's grid_sample, the noise — are fed as those f32 values). The sampled
moments (tests/golden_io.sample_idx, the golden's own sampling) are the exact-arithmetic answer that both the
reference's f32 run (the golden) and the product approximate: tests/test_gpu_dreamer.py bounds the product's
distance from them, and tools/grad_attrib.py shows the reference's. Posterior indices must equal the golden's
(no near-tie flips at these sizes), else the case is skipped.
  python tests/golden/gen_f64_moments.py [case ...]   -> tests/golden/f64/<case>.npz
  python tests/golden/gen_f64_moments.py --grads [case ...]   adds g_<tensor>__n / __s: the float64 gradients of one
      _cal_grad at the initial weights, sampled like the golden's g_* (tests/test_gpu_dreamer.py's gradient test)
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "safe-dreamer_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from golden_io import CASES, batch, initial, load_case, sample_idx  # noqa: E402
from oracle import ref_cpu  # noqa: E402


def moments(name, dt):
    """[(moments {tensor: (m, v)} float64 samples, posterior index flips vs the golden)] for updates 0 and 1"""
    ref_cpu.DT = dt
    try:
        z, cfg, spec, params, obs = load_case(name)
        ag = ref_cpu.OracleAgent(spec, params)
        cast = lambda t: t.to(dt) if torch.is_tensor(t) and t.is_floating_point() else t  # noqa: E731
        out = []
        for u in range(2):
            data = {k: cast(v) for k, v in batch(z, u, obs).items()}
            init = type(initial(z, u, spec))(cast(t) for t in initial(z, u, spec))
            (ps, _), _, _ = ag.update(data, init, int(z[f"u{u}_seed"]), keep={})
            flips = int((ps.argmax(-1).numpy() != z[f"u{u}_post_idx"]).sum())
            mom = {}
            for k in spec.shapes:
                st = ag.state[id(ag.P[k])]
                idx = sample_idx(k, ag.P[k].numel())
                mom[k] = tuple(st[s].reshape(-1).double().numpy()[idx] for s in ("exp_avg", "exp_avg_sq"))
            out.append((mom, flips))
        return out
    finally:
        ref_cpu.DT = torch.float32


def grads(name, dt):
    """{g_<tensor>__n, g_<tensor>__s}: one cal_grad at the initial weights (as the golden's g_*, gen_golden.py)"""
    ref_cpu.DT = dt
    try:
        z, cfg, spec, params, obs = load_case(name)
        ag = ref_cpu.OracleAgent(spec, params)
        cast = lambda t: t.to(dt) if torch.is_tensor(t) and t.is_floating_point() else t  # noqa: E731
        ag.update_slow_target()
        if spec.rep_loss == "dreamerpro":
            ag.ema_update()
        data = {k: cast(v) for k, v in batch(z, 0, obs).items()}
        init = type(initial(z, 0, spec))(cast(t) for t in initial(z, 0, spec))
        ag.cal_grad(data, init, int(z["u0_seed"]))
        out = {}
        for k in spec.shapes:
            g = ag.P[k].grad
            flat = (torch.zeros_like(ag.P[k]) if g is None else g).reshape(-1).double().numpy()
            out[f"g_{k}__n"] = np.asarray(np.linalg.norm(flat))
            out[f"g_{k}__s"] = flat[sample_idx(k, flat.size)]
        return out
    finally:
        ref_cpu.DT = torch.float32


def main():
    torch.set_num_threads(8)
    if sys.argv[1:2] == ["--grads"]:
        for name in sys.argv[2:] or list(CASES):
            fx = os.path.join(HERE, "f64", f"{name}.npz")
            if not os.path.exists(fx):
                continue
            arrs = dict(np.load(fx))
            arrs.update(grads(name, torch.float64))
            np.savez_compressed(fx, **arrs)
            print(f"{name}: {len(arrs)} arrays")
        return
    for name in sys.argv[1:] or list(CASES):
        res = moments(name, torch.float64)
        if any(f for _, f in res):
            print(f"{name}: posterior index flips {[f for _, f in res]} in float64: skipped")
            continue
        arrs = {f"u{u}_{k}__{w}": a for u, (mom, _) in enumerate(res) for k, (m, v) in mom.items()
                for w, a in (("m", m), ("v", v))}
        np.savez_compressed(os.path.join(HERE, "f64", f"{name}.npz"), **arrs)
        print(f"{name}: {len(arrs)} arrays")


if __name__ == "__main__":
    main()
