"""Precision variants against exact arithmetic, over every golden case (build container, CPU).

For each golden case: the reference's own f32 LaProp moments (the golden), the oracle's float64 moments
(tests/golden/gen_f64_moments.py: the same samples, images and noise in float64 — the answer every f32 evaluation
approximates) and, per variant, the product's moments dumped on the GPU box by tools/dump_opt.py. Prints per case and
variant the worst bound ratio over all tensors and both updates of
  gpu~golden  — what the golden update test asserts (<= 1 passes; tests/test_gpu_dreamer.py's bounds)
  gpu~f64     — the variant's distance from exact arithmetic, on the same bounds
beside golden~f64 (the reference's own f32 distance from exact arithmetic) and the worst tensor.
  python tools/precision_study.py <dump dir> [<dump dir> ...]   (each dir: <case>_opt_u<u>.npz per case)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "safe-dreamer_amd"),
                os.path.join(ROOT, "tests", "golden")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from gen_f64_moments import moments  # noqa: E402
from golden_io import CASES, load_case  # noqa: E402
from parity import bound_ratio  # noqa: E402


def main():
    dirs = sys.argv[1:]
    torch.set_num_threads(8)
    print(f"{'case':18s} {'variant':10s} {'gpu~golden':>10s} {'gpu~f64':>8s} {'golden~f64':>10s}  worst tensor (gpu~golden)")
    for name in CASES:
        z, _, spec, _, _ = load_case(name)
        fx = os.path.join(ROOT, "tests", "golden", "f64", f"{name}.npz")  # committed (gen_f64_moments.py), else recomputed
        if os.path.exists(fx):
            f = np.load(fx)
            f64 = [({k: (f[f"u{u}_{k}__m"], f[f"u{u}_{k}__v"]) for k in spec.shapes}, None) for u in range(2)]
        else:
            f64 = moments(name, torch.float64)
        for d in dirs:
            worst = (0.0, "", 0.0, 0.0)
            worst64 = 0.0
            ok = True
            for u in range(2):
                path = os.path.join(d, f"{name}_opt_u{u}.npz")
                if not os.path.exists(path):
                    ok = False
                    break
                gpu = np.load(path)
                for k in spec.shapes:
                    m_ref, v_ref = z[f"u{u}_st_{k}__m"].astype(np.float64), z[f"u{u}_st_{k}__v"].astype(np.float64)
                    m64, v64 = f64[u][0][k]
                    tiny = np.sqrt(v_ref) < 1e-3 * np.sqrt(v_ref).max()
                    for what, ref, x64 in (("m", m_ref, m64), ("v", v_ref, v64)):
                        g = gpu[f"{k}__{what}"].astype(np.float64)
                        if what == "v":
                            b = lambda x, y: bound_ratio(x, y, 2e-2, 2e-4 * np.abs(y).max() + 1e-30)  # noqa: E731
                        else:
                            b = lambda x, y: bound_ratio(x, y, 2e-2, 1e-2 * np.abs(y).max() + 1e-30, mask=tiny)  # noqa: E731
                        r_g, r_64, r_gold = b(g, ref), b(g, x64), b(ref, x64)
                        worst64 = max(worst64, r_64)
                        if r_g > worst[0]:
                            worst = (r_g, f"u{u} {what} {k}", r_64, r_gold)
            if not ok:
                print(f"{name:18s} {os.path.basename(d.rstrip('/')):10s} (no dump)")
                continue
            print(f"{name:18s} {os.path.basename(d.rstrip('/')):10s} {worst[0]:10.3f} {worst64:8.3f} {worst[3]:10.3f}  "
                  f"{worst[1][-60:]} (its gpu~f64 {worst[2]:.3f})", flush=True)


if __name__ == "__main__":
    main()
