"""Who is closer to exact arithmetic? (attribute the golden optimizer-bound headroom.)

For a golden case, runs the CPU oracle (oracle/ref_cpu.py, the reference's algorithm) twice over the case's two
updates: in float32 (the reference's arithmetic: it matches the golden to ~1e-3 of m) and in float64 (ref_cpu.DT;
the same discrete samples, images, augmentation and noise as inputs). The float64 LaProp moments are the answer every
f32 run approximates. Prints, per update, the tensors whose moments sit furthest from the golden for the product's
GPU run (the moments the GPU test dumps with SDREAMER_DUMP_OPT=1 into gpurun_out/golden/<case>_opt_u<u>.npz), and
for each the bound ratio (|x - y| / (atol + rtol |y|), the GPU test's bound) of:
  gpu vs golden  — what the GPU test measures
  golden vs f64  — the reference's own f32 distance from exact arithmetic
  gpu vs f64     — the product's distance from exact arithmetic
  python tools/grad_attrib.py [case] [gpu dump dir]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "safe-dreamer_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
from gen_f64_moments import moments  # noqa: E402
from golden_io import load_case  # noqa: E402
from parity import bound_ratio  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "walker_r2aug"
    gdir = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "gpurun_out", "golden")
    torch.set_num_threads(8)
    z, _, spec, _, _ = load_case(name)
    f32, f64 = moments(name, torch.float32), moments(name, torch.float64)
    print(f"{name}: posterior index flips f32 {[f for _, f in f32]}, f64 {[f for _, f in f64]} (vs the golden)")
    for u in range(2):
        path = os.path.join(gdir, f"{name}_opt_u{u}.npz")
        gpu = np.load(path) if os.path.exists(path) else None
        rows = []
        for k in spec.shapes:
            m_ref, v_ref = z[f"u{u}_st_{k}__m"].astype(np.float64), z[f"u{u}_st_{k}__v"].astype(np.float64)
            m64, v64 = f64[u][0][k]
            m32, v32 = f32[u][0][k]
            tiny = np.sqrt(v_ref) < 1e-3 * np.sqrt(v_ref).max()

            def br(x, y, what):
                if what == "v":
                    return bound_ratio(x, y, 2e-2, 2e-4 * np.abs(y).max() + 1e-30)
                return bound_ratio(x, y, 2e-2, 1e-2 * np.abs(y).max() + 1e-30, mask=tiny)
            for what, ref, x64, x32, g in (("m", m_ref, m64, m32, gpu[f"{k}__m"] if gpu is not None else None),
                                           ("v", v_ref, v64, v32, gpu[f"{k}__v"] if gpu is not None else None)):
                rows.append((br(g, ref, what) if g is not None else float("nan"), k, what, br(ref, x64, what),
                             br(x32, x64, what), br(g, x64, what) if g is not None else float("nan")))
        rows.sort(key=lambda r: -np.nan_to_num(r[0], nan=-1))
        print(f"\nupdate {u} ({'gpu dump ' + path if gpu is not None else 'no gpu dump'})")
        print(f"{'tensor':48s} mom  gpu~golden  golden~f64  oracle32~f64  gpu~f64")
        for r in rows[:8]:
            print(f"{r[1][-48:]:48s} {r[2]:3s}  {r[0]:10.3f}  {r[3]:10.3f}  {r[4]:12.3f}  {r[5]:7.3f}")


if __name__ == "__main__":
    main()
