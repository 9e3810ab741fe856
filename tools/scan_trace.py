"""Per-phase breakdown of the fused observe scan's launches (GPU box, measurement aid).

Loads the -DSD_SCAN_TRACE build of the library (safe-dreamer_amd/sdreamer/_lib_trace, `make OUT=../sdreamer/_lib_trace
BUILD=build_trace EXTRA=-DSD_SCAN_TRACE`), runs RSSM.observe forward + backward at a BASELINE config and reads the
workgroups' timestamps (s_memrealtime, 100 MHz = 10 ns ticks): per kernel, the median over steps of
  gap    = first workgroup entry - previous launch's last workgroup exit (the dependent-launch boundary)
  skew   = last workgroup entry - first workgroup entry (dispatch ramp)
  stage  = entry -> operands staged (weights issued, prologue loads, norms, LDS panel; median over workgroups)
  mma    = staged -> contraction reduced
  epi    = reduced -> exit
  span   = first entry -> last exit
  python tools/scan_trace.py [config] [B] [T] [row_tile]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("SDHIP_LIB", os.path.join(ROOT, "safe-dreamer_amd", "sdreamer", "_lib_trace", "libsdhip.so"))
sys.path[:0] = [ROOT, os.path.join(ROOT, "safe-dreamer_amd"), os.path.join(ROOT, "tests")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

TR_WG = 2048
FWD = {1: "k_hid", 2: "k_gate", 3: "k_slab(obs+x0)", 4: "k_logit_rows"}
BWD = {0: "k_dlogit", 1: "k_dgru", 2: "k_dhh", 3: "k_dhp", 4: "k_carry"}


def main():
    from test_gpu_scan import _model
    from sdreamer import rssm as R
    config = sys.argv[1] if len(sys.argv) > 1 else "dmc/cnn"
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    T = int(sys.argv[3]) if len(sys.argv) > 3 else 64
    R.SCAN_ROW_TILE = int(sys.argv[4]) if len(sys.argv) > 4 else R.SCAN_ROW_TILE
    m, embed, action, reset, init, ups = _model(config, B, T, E=1024)
    reset[:, 1:] = False
    buf = torch.zeros(2 * T * 8 * TR_WG * 4, dtype=torch.int64, device="cuda")

    def run():
        e = embed.clone().requires_grad_(True)
        st, de, lo = m.observe(e, action, init, reset, seed=1234, row_offset=0)
        ((st * ups[0]).sum() + (de * ups[1]).sum() + (lo * ups[2]).sum()).backward()
        torch.cuda.synchronize()

    for _ in range(2):
        run()
    buf.zero_()
    R.SCAN_TRACE = buf
    run()
    R.SCAN_TRACE = None
    tr = buf.view(2 * T * 8, TR_WG, 4).cpu().numpy().astype(np.int64)
    rows = {}
    prev_end = None
    order = [(t * 8 + w, "fwd", FWD[w]) for t in range(T) for w in (1, 2, 3, 4)] + \
            [((T + t) * 8 + w, "bwd", BWD[w]) for t in reversed(range(T)) for w in (0, 1, 2, 3, 4)]
    for slot, ph, name in order:
        x = tr[slot]
        used = x[:, 0] > 0
        if not used.any():
            prev_end = None
            continue
        x = x[used]
        first, last_in, end = x[:, 0].min(), x[:, 0].max(), x[:, 3].max()
        r = rows.setdefault((ph, name), {"gap": [], "skew": [], "stage": [], "mma": [], "epi": [], "span": [],
                                         "wstage": [], "wmma": [], "wepi": [], "wid": [], "wgs": int(used.sum())})
        wi = int(np.argmax(x[:, 3]))  # the workgroup that exits last: its own phases
        r["wstage"].append((x[wi, 1] - x[wi, 0]) * 10e-3)
        r["wmma"].append((x[wi, 2] - x[wi, 1]) * 10e-3)
        r["wepi"].append((x[wi, 3] - x[wi, 2]) * 10e-3)
        r["wid"].append(int(np.flatnonzero(used)[wi]))
        if prev_end is not None:
            r["gap"].append((first - prev_end) * 10e-3)
        r["skew"].append((last_in - first) * 10e-3)
        r["stage"].append(np.median(x[:, 1] - x[:, 0]) * 10e-3)
        r["mma"].append(np.median(x[:, 2] - x[:, 1]) * 10e-3)
        r["epi"].append(np.median(x[:, 3] - x[:, 2]) * 10e-3)
        r["span"].append((end - first) * 10e-3)
        prev_end = end
    print(f"scan phase breakdown: {config} B{B} T{T} row_tile {R.SCAN_ROW_TILE or 16} (us, median over steps)")
    print(f"{'phase':4s} {'kernel':16s} {'WGs':>5s} {'gap':>6s} {'skew':>6s} {'stage':>6s} {'mma':>6s} {'epi':>6s} "
          f"{'span':>6s} | last-exiting WG: {'stage':>6s} {'mma':>6s} {'epi':>6s} {'id (mode)':>9s}")
    tot = {"fwd": 0.0, "bwd": 0.0}
    for (ph, name), r in rows.items():
        med = {k: (float(np.median(v)) if v else float("nan")) for k, v in r.items() if k not in ("wgs", "wid")}
        ids, cnt = np.unique(np.array(r["wid"]), return_counts=True)
        wid_mode = int(ids[np.argmax(cnt)])
        tot[ph] += med["span"] + (med["gap"] if med["gap"] == med["gap"] else 0.0)
        print(f"{ph:4s} {name:16s} {r['wgs']:5d} {med['gap']:6.2f} {med['skew']:6.2f} {med['stage']:6.2f} "
              f"{med['mma']:6.2f} {med['epi']:6.2f} {med['span']:6.2f} |                  {med['wstage']:6.2f} "
              f"{med['wmma']:6.2f} {med['wepi']:6.2f} {wid_mode:9d}")
    print(f"per step: forward {tot['fwd']:.2f} us, backward {tot['bwd']:.2f} us (span + gap medians)")


if __name__ == "__main__":
    main()
