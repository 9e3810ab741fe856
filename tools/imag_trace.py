"""Per-phase breakdown of the fused imagination's launches (GPU box, measurement aid), as tools/scan_trace.py does
for the observe scan: the -DSD_SCAN_TRACE build of the library, one eager update of the bench workload, and per launch
of an imagination step the median over steps of gap / skew / stage (entry -> operands staged: row-norm partials, the
one-hot index search) / mma (staged -> main loop done) / epi / span, in us.
  python tools/imag_trace.py [config]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("SDHIP_LIB", os.path.join(ROOT, "safe-dreamer_amd", "sdreamer", "_lib_trace", "libsdhip.so"))
sys.path[:0] = [ROOT, os.path.join(ROOT, "safe-dreamer_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from bench import WORKLOADS, _Sp, _Spaces, synth_buffer  # noqa: E402

TR_WG = 2048
NAMES = {0: "k_onehot_lin", 1: "k_rmslin(a1)", 2: "k_rmslin(a2)", 3: "k_rmslin(a3)", 4: "k_action", 5: "k_hid",
         6: "k_gate", 7: "k_lin", 8: "k_rmslin(i1)", 9: "k_rmslin(i2)", 10: "k_rmslin(i3)", 12: "k_prior"}


def main():
    from sdreamer import dreamer as DR
    from sdreamer.config import load_config
    config = sys.argv[1] if len(sys.argv) > 1 else "dmc/cnn"
    A, discrete, _ = WORKLOADS[config]
    cfg = load_config(config, ["device=cuda:0", "model.compile=False"])
    torch.manual_seed(0)
    act = _Sp((A,))
    if discrete:
        act.discrete = True
    ag = DR.Dreamer(cfg.model, _Spaces({"image": _Sp((64, 64, 3))}), act)
    ag.use_graphs = False
    ag.use_side_stream = False  # the imagination alone on the stream: launch gaps are its own
    L, H1 = int(cfg.batch_length), int(cfg.model.imag_horizon) + 1
    buf = synth_buffer(cfg, torch.device("cuda:0"), 0, T=max(160, 2 * (L + 1)), A=A, discrete=discrete)
    for _ in range(2):
        ag.update(buf)
    trace = torch.zeros(H1 * 16 * TR_WG * 4, dtype=torch.int64, device="cuda")
    DR.IMAG_TRACE = trace
    ag.update(buf)
    torch.cuda.synchronize()
    DR.IMAG_TRACE = None
    tr = trace.view(H1 * 16, TR_WG, 4).cpu().numpy().astype(np.int64)
    rows, prev_end = {}, None
    for t in range(H1):
        for k in range(16):
            x = tr[t * 16 + k]
            used = x[:, 0] > 0
            if not used.any():
                continue
            x = x[used]
            first, last_in, end = x[:, 0].min(), x[:, 0].max(), x[:, 3].max()
            r = rows.setdefault(k, {"gap": [], "skew": [], "stage": [], "mma": [], "epi": [], "span": [],
                                    "wgs": int(used.sum())})
            if prev_end is not None:
                r["gap"].append((first - prev_end) * 10e-3)
            r["skew"].append((last_in - first) * 10e-3)
            r["stage"].append(np.median(x[:, 1] - x[:, 0]) * 10e-3)
            r["mma"].append(np.median(x[:, 2] - x[:, 1]) * 10e-3)
            r["epi"].append(np.median(x[:, 3] - x[:, 2]) * 10e-3)
            r["span"].append((end - first) * 10e-3)
            prev_end = end
    print(f"imagination phase breakdown: {config} N={ag.batch_size * L if hasattr(ag, 'batch_size') else ''} "
          f"H1={H1} (us, median over steps; WGs recorded up to {TR_WG})")
    print(f"{'kernel':14s} {'WGs':>5s} {'gap':>6s} {'skew':>6s} {'stage':>6s} {'mma':>6s} {'epi':>6s} {'span':>6s}")
    tot = 0.0
    for k in sorted(rows):
        r = rows[k]
        med = {kk: (float(np.median(v)) if v else float("nan")) for kk, v in r.items() if kk != "wgs"}
        tot += med["span"] + (med["gap"] if med["gap"] == med["gap"] else 0.0)
        print(f"{NAMES.get(k, str(k)):14s} {r['wgs']:5d} {med['gap']:6.2f} {med['skew']:6.2f} {med['stage']:6.2f} "
              f"{med['mma']:6.2f} {med['epi']:6.2f} {med['span']:6.2f}")
    print(f"per step: {tot:.2f} us (span + gap medians)")


if __name__ == "__main__":
    main()
