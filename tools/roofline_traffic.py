"""HBM traffic per launch of the bench's roofline kernels from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE).

Selects each kernel's dispatches by name and grid, averages per dispatch, applies the gfx950 correction from
MI355X_MICROARCH.md (FETCH_SIZE reports half of the bytes of wide coalesced reads: x2), converts KB -> bytes and
writes one JSON keyed like bench.py's roofline entries (`key`), with each kernel's algorithmic bytes per launch
(every operand read once, every output written once) at the walker B16 L64 H15 workload:
  N = B*L = 1,024 imagination rows, D = 2,048, U = 256, Dg = D / 8 = 256; encoder stage 2 at 1,024 images.
Usage: python tools/roofline_traffic.py <fetch.db> <write.db> <out.json>"""
import json
import sqlite3
import sys

N, D, U, DG = 1024, 2048, 256, 256
KERNELS = {  # key: (name substring of the demangled symbol, grid filter (wg_x, wg_y, wg_z) or None, algorithmic bytes)
    "k_lin": ("k_lin<32, 32>", (U // 32, N // 32, 3),
              4.0 * (N * D + 3 * U * D + 3 * N * U + 2 * (U // 16) * N)),  # deter' + 3 W + 3 outputs + row partials
    "k_hid": ("k_hid(sd_imagine", None,
              4.0 * (N * D + 3 * N * U + D * (DG + 3 * U) + N * D + N * D // 64)),  # h, x0/x1/x2, W, hp, partials
    "k_gate": ("k_gate(sd_imagine", None, 4.0 * (N * D + 3 * D * DG + 2 * N * D)),  # hp, W, hold, deter'
    # NHWC input read once + pooled (f32) + y (f32) + argmax (u8) + rstd (f32 per pooled pixel) written once
    "conv_fwd_direct_pool": ("conv_fwd_direct_pool<48", (8192, 1, 1),
                             4.0 * 1024 * 32 * 32 * 32 + 1024 * 16 * 16 * (48 * (4 + 4 + 1) + 4)),
}


def per_launch(path, counter, name_like, grid):
    db = sqlite3.connect(path)
    cols = [r[1] for r in db.execute("pragma table_info(counters_collection)")]
    gz = "grid_size_z" if "grid_size_z" in cols else "1"
    rows = db.execute(f"select grid_size_x, grid_size_y, {gz}, workgroup_size_x, value from counters_collection "
                      "where counter_name = ? and kernel_name like ?", (counter, f"%{name_like}%")).fetchall()
    vals = [v for gx, gy, gzv, wx, v in rows if grid is None or (gx // max(wx, 1), gy, gzv) == tuple(grid)]
    return (sum(vals) / len(vals) if vals else None), len(vals)


def main(fetch_db, write_db, out):
    res = {}
    kb = 1024.0  # rocprofv3 FETCH_SIZE / WRITE_SIZE are in kilobytes
    for key, (name, grid, algo) in KERNELS.items():
        f, nf = per_launch(fetch_db, "FETCH_SIZE", name, grid)
        w, nw = per_launch(write_db, "WRITE_SIZE", name, grid)
        r = {"kernel": name, "grid_workgroups": grid, "algorithmic_bytes": algo, "dispatches": [nf, nw],
             "fetch_bytes_raw": f * kb if f is not None else None,
             "fetch_bytes": 2 * f * kb if f is not None else None,  # gfx950: FETCH_SIZE = 1/2 of wide reads
             "write_bytes": w * kb if w is not None else None}
        r["traffic_bytes"] = (r["fetch_bytes"] or 0) + (r["write_bytes"] or 0) if f is not None else None
        r["traffic_over_algorithmic"] = r["traffic_bytes"] / algo if r["traffic_bytes"] else None
        res[key] = r
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:4])
