"""GPU box: the golden cases' two product updates with the current environment (e.g. SDREAMER_CONV6=s2, the encoder's
second stage forward on bf16x6), their sampled LaProp moments dumped as tools/grad_attrib.py reads them — no
assertions, so a variant that leaves a golden bound can still be compared against float64.
  python tools/dump_opt.py <out dir> [case ...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "safe-dreamer_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from golden_io import CASES, batch, initial  # noqa: E402
from test_gpu_dreamer import _opt_samples, build_agent  # noqa: E402


def main():
    out = sys.argv[1]
    names = sys.argv[2:] or list(CASES)
    os.makedirs(out, exist_ok=True)
    for name in names:
        ag, z, spec, obs = build_agent(name)
        for u in range(2):
            data = batch(z, u, obs, "cuda")
            if "image" in obs:
                data["image"] = torch.from_numpy(z[f"u{u}_in_image"]).to("cuda")
            ag.update_batch(data, initial(z, u, spec, "cuda"), int(z[f"u{u}_seed"]))
            torch.cuda.synchronize()
            opt = _opt_samples(ag, spec)
            np.savez(os.path.join(out, f"{name}_opt_u{u}.npz"),
                     **{f"{k}__{w}": a for k, (m_, v_) in opt.items() for w, a in (("m", m_), ("v", v_))})
        print(name, "dumped", flush=True)


if __name__ == "__main__":
    main()
